"""HIP path vs the oracle / golden vectors, through the C ABI (ctypes).

Tolerances: gather bit-exact; encoders and scores normwise ||a-b||/||b||
<= TOL = 1e-5 per output vector. SURVEY §8d / the north star allow 1e-3
(SPEC_TOL); the kernels land at 2-5e-7 against the fp32 golden and the fp64
oracle, so the assertions sit at 1e-5 (round 6): a lost split plane or a
wrong scale (errors of 1e-4 and up) fails them.
"""
import ctypes

import numpy as np
import pytest
import torch

from oracle import nrms_oracle as O
from oracle import weights as W

pytestmark = pytest.mark.gpu

SPEC_TOL = 1e-3   # SURVEY §8d / north_star: "within 1e-3 rel fp32"
TOL = 1e-5        # what the assertions hold the kernels to (observed 2-5e-7)


def _module(state, V, device, **knobs):
    from newsrecommendationsystem_amd import NRMS, NRMSConfig

    class Cfg(NRMSConfig):
        num_words = V
    for k, v in knobs.items():
        setattr(Cfg, k, v)
    m = NRMS(Cfg)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in state.items()})
    return m.to(device).eval()


def _np(t):
    return t.detach().float().cpu().numpy()


@pytest.fixture(scope="module")
def gold_model(golden, golden_state, device):
    return _module(golden_state, int(golden["V"]), device)


def test_library_loads_native():
    from newsrecommendationsystem_amd import _native as N
    assert N.load().nrms_abi_version() == N.ABI_VERSION


def test_gather_bit_exact_golden(golden, golden_state, device):
    from newsrecommendationsystem_amd import _native as N
    tab = torch.from_numpy(golden_state["news_encoder.word_embedding.weight"]).to(device)
    ids = torch.from_numpy(golden["gather_ids"].astype(np.int64)).to(device)
    out = torch.empty(ids.numel(), tab.shape[1], device=device)
    N.call("nrms_embedding_gather", N.ptr(ids), ids.numel(), N.ptr(tab), tab.shape[0], tab.shape[1],
           N.ptr(out), N.stream_handle(device))
    got = _np(out).reshape(golden["gather_out"].shape)
    assert np.array_equal(got.view(np.uint32), golden["gather_out"].view(np.uint32))


@pytest.mark.parametrize("V", [70976, 1 << 20])
def test_gather_bit_exact_large(device, V):
    from newsrecommendationsystem_amd import _native as N
    g = torch.Generator(device="cpu").manual_seed(V)
    tab = torch.randn(V, 300, generator=g).to(device)
    ids = torch.randint(0, V, (4099, 20), generator=g)
    ids[0, :] = 0
    ids[1, :] = V - 1
    ids = ids.to(device)
    out = torch.empty(ids.numel(), 300, device=device)
    N.call("nrms_embedding_gather", N.ptr(ids), ids.numel(), N.ptr(tab), V, 300, N.ptr(out),
           N.stream_handle(device))
    assert torch.equal(out.view(-1, 20, 300), tab[ids])


def test_gather_bad_id_is_nan_not_fault(device):
    from newsrecommendationsystem_amd import _native as N
    tab = torch.randn(64, 300, device=device)
    ids = torch.tensor([0, 63, 64, -1, 5], device=device)
    out = torch.empty(5, 300, device=device)
    N.call("nrms_embedding_gather", N.ptr(ids), 5, N.ptr(tab), 64, 300, N.ptr(out),
           N.stream_handle(device))
    o = _np(out)
    assert np.isnan(o[2]).all() and np.isnan(o[3]).all()
    assert np.array_equal(o[[0, 1, 4]], _np(tab)[[0, 63, 5]])


@pytest.mark.parametrize("mode", [1, 2, "cached"])
def test_news_vectors_golden(golden, golden_state, device, mode, gemm_mode):
    knobs = {"hip_cache_folded_table": mode == "cached"}
    if mode != "cached":
        knobs["hip_proj_mode"] = mode
    m = _module(golden_state, int(golden["V"]), device, **knobs)
    with torch.no_grad():
        out = _np(m.get_news_vector({"title": torch.from_numpy(golden["news_ids"].astype(np.int64))}))
    err = O.normwise_rel_err(out, golden["news_out"])
    assert err.max() < TOL, err.max()


def test_user_vectors_golden(golden, gold_model, gemm_mode):
    u_in = W.normal(int(golden["seed"]), 30, (8, 50, 300), 0.3)
    for b, n in enumerate(golden["user_len"]):
        u_in[b, : 50 - n] = 0.0
    with torch.no_grad():
        out = _np(gold_model.get_user_vector(torch.from_numpy(u_in)))
    assert O.normwise_rel_err(out, golden["user_out"]).max() < TOL


def test_user_vectors_noncontiguous_input(golden, gold_model, device):
    # evaluate.py:220-224 passes a transpose(0, 1) view
    u_in = W.normal(int(golden["seed"]), 30, (8, 50, 300), 0.3)
    for b, n in enumerate(golden["user_len"]):
        u_in[b, : 50 - n] = 0.0
    x = torch.from_numpy(u_in).to(device).transpose(0, 1).contiguous().transpose(0, 1)
    assert not x.is_contiguous()
    with torch.no_grad():
        out = _np(gold_model.get_user_vector(x))
    assert O.normwise_rel_err(out, golden["user_out"]).max() < TOL


def test_user_encode_strided_views_through_c_abi(golden, gold_model, device, gemm_mode):
    """nrms_user_encode (ABI 2) reads [B, N, D] views in place: the
    transpose(0, 1) of src/evaluate.py:220-224 (stride_b = D, stride_n = B*D)
    and a history slice of a wider tensor. Each equals the contiguous call
    bitwise and the golden user_out within TOL; no copy is made."""
    from newsrecommendationsystem_amd import _native as N
    u_in = W.normal(int(golden["seed"]), 30, (8, 50, 300), 0.3)
    for b, n in enumerate(golden["user_len"]):
        u_in[b, : 50 - n] = 0.0
    B, Nn, D = u_in.shape
    contig = torch.from_numpy(u_in).to(device)
    tview = contig.transpose(0, 1).contiguous().transpose(0, 1)   # [B, N, D], strides (D, B*D, 1)
    wide = torch.zeros(B, Nn + 7, D, device=device)
    wide[:, 7:] = contig
    sview = wide[:, 7:]                                            # strides ((N+7)*D, D, 1)
    w, keep = gold_model.user_encoder.weights()
    lib = N.load()
    nb = lib.nrms_user_encode_workspace_size(B, Nn, D)
    ws = torch.empty(nb, dtype=torch.uint8, device=device)
    outs = []
    for x in (contig, tview, sview):
        out = torch.empty(B, D, device=device)
        N.call("nrms_user_encode", N.ptr(x), B, Nn, x.stride(0), x.stride(1), ctypes.byref(w),
               N.ptr(out), N.ptr(ws), nb, N.stream_handle(device))
        outs.append(out)
    assert tview.stride() == (D, B * D, 1) and sview.stride() == ((Nn + 7) * D, D, 1)
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
    assert O.normwise_rel_err(_np(outs[1]), golden["user_out"]).max() < TOL
    # the module path hands the view over as is (bitwise the same as the C call)
    with torch.no_grad():
        assert torch.equal(gold_model.get_user_vector(tview), outs[1])
    # bad strides are rejected, not misread
    assert lib.nrms_user_encode(N.ptr(contig), B, Nn, -1, D, ctypes.byref(w), N.ptr(outs[0]),
                                N.ptr(ws), nb, N.stream_handle(device)) == N.NRMS_ERR_INVALID_ARG
    assert lib.nrms_user_encode(N.ptr(contig), B, Nn, Nn * D, D + 1, ctypes.byref(w),
                                N.ptr(outs[0]), N.ptr(ws), nb,
                                N.stream_handle(device)) == N.NRMS_ERR_UNSUPPORTED


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_forward_golden(golden, golden_state, device, mode, gemm_mode):
    m = _module(golden_state, int(golden["V"]), device, hip_proj_mode=mode)
    cand = golden["fwd_cand"].astype(np.int64)
    clk = golden["fwd_clicked"].astype(np.int64)
    with torch.no_grad():
        y = _np(m([{"title": torch.from_numpy(cand[:, i])} for i in range(cand.shape[1])],
                  [{"title": torch.from_numpy(clk[:, i])} for i in range(clk.shape[1])]))
    ref = golden["fwd_out"]
    assert np.abs(y - ref).max() <= TOL * np.abs(ref).max()
    assert O.normwise_rel_err(y, ref).max() < TOL


def test_prediction_golden(golden, gold_model, device):
    s = int(golden["seed"])
    nv = torch.from_numpy(W.normal(s, 50, (7, 300), 0.5)).to(device)
    uv = torch.from_numpy(W.normal(s, 51, (300,), 0.5)).to(device)
    with torch.no_grad():
        out = _np(gold_model.get_prediction(nv, uv))
    assert out.shape == (7,)
    assert np.abs(out - golden["pred_out"]).max() <= TOL * np.abs(golden["pred_out"]).max()


def test_raw_exp_overflow_nan(golden, golden_state, device, gemm_mode):
    sd = dict(golden_state)
    for k in ("W_Q", "W_K"):
        key = f"news_encoder.multihead_self_attention.{k}.weight"
        sd[key] = (sd[key] * golden["overflow_scale"]).astype(np.float32)
    for mode in (1, 2):
        m = _module(sd, int(golden["V"]), device, hip_proj_mode=mode, hip_cache_folded_table=False)
        with torch.no_grad():
            out = _np(m.get_news_vector({"title": torch.from_numpy(golden["news_ids"].astype(np.int64))}))
        ref = golden["overflow_out"]
        nan_ref = np.isnan(ref).any(axis=1)
        nan_got = np.isnan(out).any(axis=1)
        # rows whose max score sits within float rounding of the exp overflow
        # threshold may flip; the golden has none that close (checked below)
        assert np.array_equal(nan_ref, nan_got)
        assert np.array_equal(np.isnan(out), np.isnan(ref))
        assert O.normwise_rel_err(out[~nan_ref], ref[~nan_ref]).max() < TOL


def test_raw_exp_underflow_zero(golden, golden_state, device, gemm_mode):
    sd = dict(golden_state)
    pre = "news_encoder.multihead_self_attention"
    b = golden["underflow_bias"]
    sd[f"{pre}.W_Q.bias"] = np.full(300, b, np.float32)
    sd[f"{pre}.W_K.bias"] = np.full(300, -b, np.float32)
    sd[f"{pre}.W_Q.weight"] = np.zeros((300, 300), np.float32)
    sd[f"{pre}.W_K.weight"] = np.zeros((300, 300), np.float32)
    m = _module(sd, int(golden["V"]), device)
    with torch.no_grad():
        out = _np(m.get_news_vector({"title": torch.from_numpy(golden["news_ids"].astype(np.int64))}))
    assert np.array_equal(out, golden["underflow_out"])


def test_out_of_range_ids_raise(gold_model, golden):
    V = int(golden["V"])
    with pytest.raises(IndexError):
        gold_model.get_news_vector({"title": torch.tensor([[0, V]])})
    with pytest.raises(IndexError):
        gold_model.get_news_vector({"title": torch.tensor([[-1, 3]])})


def test_train_mode_forward_matches_hip_eval(golden, golden_state, device):
    """Training mode (ATen autograd, dropout p=0) and the HIP eval path agree."""
    V = int(golden["V"])
    m = _module(golden_state, V, device, dropout_probability=0.0)
    cand = torch.from_numpy(golden["fwd_cand"].astype(np.int64))
    clk = torch.from_numpy(golden["fwd_clicked"].astype(np.int64))
    ev = _np(m.forward_ids(cand, clk))
    m.train()
    tr = m.forward_ids(cand, clk)
    assert tr.requires_grad
    assert np.abs(_np(tr) - ev).max() / np.abs(ev).max() < 1e-5


@pytest.mark.parametrize("L", [1, 5, 20, 32, 50, 64, 65, 130])
def test_news_encoder_title_lengths_vs_oracle(device, L):
    V = 512
    sd = W.nrms_state(7, V)
    m = _module(sd, V, device, hip_cache_folded_table=False)
    ids = W.titles(7, 300 + L, 33, V, L=L, min_len=1)
    with torch.no_grad():
        out = _np(m.get_news_vector({"title": torch.from_numpy(ids)}))
    ref = O.news_encode(ids, sd, np.float64)
    assert O.normwise_rel_err(out, ref).max() < TOL


@pytest.mark.parametrize("L", [5, 20, 32, 50])
def test_news_encoder_cached_folded_table_title_lengths(device, L):
    """The eval path with the default cached folded table (rows of
    nrms_qkv_row_stride) at title lengths the fused kernel does not take:
    the stage kernels read the padded rows (L != 20 used to fail)."""
    V = 512
    sd = W.nrms_state(7, V)
    m = _module(sd, V, device)
    assert getattr(m.config, "hip_cache_folded_table", True)
    ids = W.titles(7, 700 + L, 29, V, L=L, min_len=1)
    with torch.no_grad():
        out = _np(m.get_news_vector({"title": torch.from_numpy(ids)}))
        again = _np(m.get_news_vector({"title": torch.from_numpy(ids)}))   # cached table reused
    ref = O.news_encode(ids, sd, np.float64)
    assert O.normwise_rel_err(out, ref).max() < TOL
    assert np.array_equal(out, again)


def test_empty_batch(gold_model):
    with torch.no_grad():
        out = gold_model.get_news_vector({"title": torch.zeros(0, 20, dtype=torch.long)})
    assert tuple(out.shape) == (0, 300)


@pytest.mark.parametrize("B,C,N", [(1, 1, 1), (3, 5, 50), (37, 5, 50), (5, 2, 7)])
def test_forward_shapes_vs_oracle(device, B, C, N, gemm_mode):
    V = 4096
    sd = W.nrms_state(11, V)
    m = _module(sd, V, device)
    cand, clk, _ = W.impressions(11, 500 + B, B, V, C=C, N=N)
    with torch.no_grad():
        y = _np(m.forward_ids(torch.from_numpy(cand), torch.from_numpy(clk)))
    ref = O.forward(cand, clk, sd, np.float64)
    assert y.shape == (B, C)
    assert np.abs(y - ref).max() <= TOL * max(np.abs(ref).max(), 1e-6)


def test_full_vocab_forward_vs_oracle(device):
    """BASELINE configs' vocabulary (V = 70,976) at a batch the oracle finishes
    in seconds."""
    V = 70976
    sd = W.nrms_state(3, V)
    m = _module(sd, V, device)
    cand, clk, _ = W.impressions(3, 900, 8, V)
    with torch.no_grad():
        y_f = _np(m.forward_ids(torch.from_numpy(cand), torch.from_numpy(clk), proj_mode=2))
        y_d = _np(m.forward_ids(torch.from_numpy(cand), torch.from_numpy(clk), proj_mode=1))
    ref = O.forward(cand, clk, sd, np.float64)
    for y in (y_f, y_d):
        assert np.abs(y - ref).max() <= TOL * np.abs(ref).max()


@pytest.mark.parametrize("n", [1, 3, 4, 5, 4099])
def test_fused_news_tail_vs_stages(device, n, gemm_mode):
    """Fused tail == separate stage kernels (within fp32 reordering), including
    partial last blocks (n % 4 != 0), through both id arrays."""
    from newsrecommendationsystem_amd import _native as N
    V = 1000
    sd = W.nrms_state(21, V)
    m = _module(sd, V, device, hip_cache_folded_table=False)
    ne = m.news_encoder
    qkv = ne.folded_table()                     # rows of nrms_qkv_row_stride
    packed = qkv[:, :900].contiguous()          # the stage kernels' packed layout
    assert qkv.shape[1] == N.load().nrms_qkv_row_stride(300) == 900
    ids = torch.from_numpy(W.titles(21, 40 + n, n, V, min_len=1)).to(device)
    na = n // 2
    # a NULL first id array means "identity rows" in the ABI, so never pass an empty one
    ia, ib = (ids[:na].contiguous() if na else ids), ids[na:].contiguous()
    w, keep = ne.weights()
    st = N.stream_handle(device)
    out = torch.empty(n, 300, device=device)
    nb = N.load().nrms_news_attention_pool_workspace_size(n, 20, 300)
    ws = torch.empty(nb, dtype=torch.uint8, device=device)
    N.call("nrms_news_attention_pool", N.ptr(qkv), qkv.shape[1], V, N.ptr(ia), na, N.ptr(ib), n, 20,
           ctypes.byref(w), N.ptr(out), N.ptr(ws), nb, st)
    out900 = torch.empty(n, 300, device=device)     # same rows at stride 900: bitwise equal
    N.call("nrms_news_attention_pool", N.ptr(packed), 900, V, N.ptr(ia), na, N.ptr(ib), n, 20,
           ctypes.byref(w), N.ptr(out900), N.ptr(ws), nb, st)
    assert torch.equal(out, out900)
    ctx = torch.empty(n * 20, 300, device=device)
    sc = torch.empty(n * 20, device=device)
    ref = torch.empty(n, 300, device=device)
    N.call("nrms_self_attention", N.ptr(packed), V, N.ptr(ia), na, N.ptr(ib), n, 20, ctypes.byref(w),
           N.ptr(ctx), st)
    N.call("nrms_additive_attention", N.ptr(ctx), n, 20, ctypes.byref(w), N.ptr(sc), N.ptr(ref), st)
    err = ((out - ref).norm(dim=1) / ref.norm(dim=1)).max()
    assert err < 1e-5, float(err)
    oracle = O.news_encode(ids.cpu().numpy(), sd, np.float64)
    assert O.normwise_rel_err(_np(out), oracle).max() < TOL


def test_full_size_properties(device, gemm_mode):
    """BASELINE config 3 (B = 1024, 1+K = 5, 50 clicked, V = 70,976): size-
    independent properties — folded == direct within fp32 rounding, sharding
    the batch changes nothing (each impression depends only on its own rows),
    repeated calls are bitwise deterministic."""
    V = 70976
    sd = W.nrms_state(5, V)
    m = _module(sd, V, device)
    cand, clk, _ = W.impressions(5, 1000, 1024, V)
    c, k = torch.from_numpy(cand), torch.from_numpy(clk)
    with torch.no_grad():
        y1 = m.forward_ids(c, k, proj_mode=2)
        y2 = m.forward_ids(c, k, proj_mode=2)
        yd = m.forward_ids(c, k, proj_mode=1)
        halves = torch.cat([m.forward_ids(c[:512], k[:512], proj_mode=2),
                            m.forward_ids(c[512:], k[512:], proj_mode=2)])
    assert torch.isfinite(y1).all()
    assert torch.equal(y1, y2)
    assert torch.equal(y1, halves)
    rel = (y1 - yd).norm() / y1.norm()
    assert rel < 1e-5, float(rel)


def test_stage_abi_matches_module(golden, golden_state, device):
    """The per-stage entry points compose to the same news vectors (split-bf16
    x6: the staged projection and the module's pre-split one agree bitwise)."""
    from newsrecommendationsystem_amd import _native as N
    with N.gemm_arith(N.NRMS_GEMM_SPLIT_BF16X6):
        _stage_abi_matches_module(golden, golden_state, device)


def _stage_abi_matches_module(golden, golden_state, device):
    from newsrecommendationsystem_amd import _native as N
    m = _module(golden_state, int(golden["V"]), device, hip_cache_folded_table=False,
                hip_proj_mode=1)
    ne = m.news_encoder
    ids = torch.from_numpy(golden["news_ids"].astype(np.int64)).to(device)
    n, L = ids.shape
    tab = ne.table()
    w, keep = ne.weights()
    st = N.stream_handle(device)
    qkv = torch.empty(n * L, 900, device=device)
    ctx = torch.empty(n * L, 300, device=device)
    sc = torch.empty(n * L, device=device)
    out = torch.empty(n, 300, device=device)
    N.call("nrms_qkv_project", N.ptr(tab), tab.shape[0], N.ptr(ids), n * L, ctypes.byref(w),
           N.ptr(qkv), 0, st)
    N.call("nrms_self_attention", N.ptr(qkv), n * L, None, n, None, n, L, ctypes.byref(w),
           N.ptr(ctx), st)
    N.call("nrms_additive_attention", N.ptr(ctx), n, L, ctypes.byref(w), N.ptr(sc), N.ptr(out), st)
    with torch.no_grad():
        ref = m.get_news_vector({"title": ids.cpu()})   # fused tail kernel
    assert (out - ref).norm() / ref.norm() < 1e-6
    # the fused entry point on the same projected rows
    fused = torch.empty(n, 300, device=device)
    nb = N.load().nrms_news_attention_pool_workspace_size(n, L, 300)
    ws = torch.empty(nb, dtype=torch.uint8, device=device)
    N.call("nrms_news_attention_pool", N.ptr(qkv), 0, n * L, None, n, None, n, L, ctypes.byref(w),
           N.ptr(fused), N.ptr(ws), nb, st)
    # (no ids given: every token its own row) bitwise the module's path with
    # token compaction off, and to fp32 rounding with it on
    lib = N.load()
    prev = lib.nrms_set_token_compaction(0)
    try:
        with torch.no_grad():
            ref0 = m.get_news_vector({"title": ids.cpu()})
    finally:
        lib.nrms_set_token_compaction(prev)
    assert torch.equal(fused, ref0)
    assert (fused - ref).norm() / ref.norm() < 2e-6
    assert O.normwise_rel_err(_np(fused), golden["news_out"]).max() < TOL
    # stage 1 alone against the oracle's projection
    x = golden_state["news_encoder.word_embedding.weight"][golden["news_ids"].astype(np.int64)]
    p = "news_encoder.multihead_self_attention"
    qkv_ref = np.concatenate([O.linear(x.reshape(-1, 300), golden_state[f"{p}.{n_}.weight"],
                                       golden_state[f"{p}.{n_}.bias"], np.float64)
                              for n_ in ("W_Q", "W_K", "W_V")], axis=1)
    assert O.normwise_rel_err(_np(qkv), qkv_ref).max() < 1e-5


@pytest.mark.parametrize("case", ["table", "table_ld900", "gather_bad_ids", "tiny", "vocab"])
def test_qkv_project_ws_vs_staged_gemm(device, gemm_mode, case):
    """nrms_qkv_project_ws (W split once per call, A tile resident in LDS:
    proj_x6.hip) against nrms_qkv_project (the staged GEMM): bitwise the same
    rows under x6 (and f32, where both are the staged GEMM); under f16x3 (the
    kernel's scaled split-f16 arithmetic) within 2e-6 of the fp64 oracle per
    row, as the staged rows. NaN rows for invalid ids, row counts off the
    64-row tile, the unpadded 900-float stride."""
    from newsrecommendationsystem_amd import _native as N
    g = torch.Generator(device="cpu").manual_seed(11)
    m = _module(W.nrms_state(5, 64), 64, device)
    w, keep = m.news_encoder.weights()
    V = {"table": 3013, "table_ld900": 3013, "gather_bad_ids": 500, "tiny": 37, "vocab": 70976}[case]
    X = (torch.randn(V, 300, generator=g) * 0.5).to(device)
    ids = None
    M = V
    if case == "gather_bad_ids":
        idt = torch.randint(0, V, (137 * 20,), generator=g)
        idt[5], idt[77], idt[1000] = -1, V, 0
        ids = idt.to(device)
        M = ids.numel()
    if case == "tiny":
        M = 5
    ld = 900 if case == "table_ld900" else N.load().nrms_qkv_row_stride(300)
    st = N.stream_handle(device)
    ref = torch.full((M, ld), 7.0, device=device)
    got = torch.full((M, ld), 7.0, device=device)
    N.call("nrms_qkv_project", N.ptr(X), V, N.ptr(ids) if ids is not None else None, M, ctypes.byref(w),
           N.ptr(ref), ld, st)
    nb = N.load().nrms_qkv_project_workspace_size(300)
    wsb = torch.empty(nb, dtype=torch.uint8, device=device)
    N.call("nrms_qkv_project_ws", N.ptr(X), V, N.ptr(ids) if ids is not None else None, M, ctypes.byref(w),
           N.ptr(got), ld, N.ptr(wsb), nb, st)
    torch.cuda.synchronize()
    if gemm_mode != "f16x3":
        assert torch.equal(got.view(torch.int32), ref.view(torch.int32))
    else:
        xa = X.cpu().numpy().astype(np.float64)
        ia = np.arange(M) if ids is None else ids.cpu().numpy()
        ok = (ia >= 0) & (ia < V)
        sd = W.nrms_state(5, 64)
        p = "news_encoder.multihead_self_attention"
        want = np.concatenate([O.linear(xa[ia[ok]], sd[f"{p}.{n_}.weight"], sd[f"{p}.{n_}.bias"], np.float64)
                               for n_ in ("W_Q", "W_K", "W_V")], axis=1)
        g_ok, r_ok = _np(got[:, :900])[ok], _np(ref[:, :900])[ok]
        assert O.normwise_rel_err(g_ok, want).max() < 2e-6
        assert O.normwise_rel_err(r_ok, want).max() < 2e-6
        assert torch.isnan(got[torch.from_numpy(~ok).to(device), :900]).all()
    if case == "gather_bad_ids":
        assert torch.isnan(got[[5, 77], :900]).all() and not torch.isnan(got[1000]).any()
    assert (got[:, 900:] == 7.0).all()   # the row padding is not written


@pytest.mark.parametrize("M", [300, 20001])
def test_qkv_project_f16x3_range(device, M):
    """The f16x3 projection's power-of-two scaling (proj_x6.hip): A rows from
    1e-20 to 1e30 in magnitude (beyond fp16's range both ways) against W_Q
    scaled by 1e5 and W_K by 1e-8 project within 2e-6 of the fp64 oracle per
    row and per Q / K / V segment; an all-zero row gives exactly the bias, a
    row holding an inf gives NaN; at M = 300 and at M = 20,001 (313 row
    tiles, a partial last one)."""
    from newsrecommendationsystem_amd import _native as N
    sd = dict(W.nrms_state(5, 64))
    p = "news_encoder.multihead_self_attention"
    sd[f"{p}.W_Q.weight"] = (sd[f"{p}.W_Q.weight"] * np.float32(1e5)).astype(np.float32)
    sd[f"{p}.W_K.weight"] = (sd[f"{p}.W_K.weight"] * np.float32(1e-8)).astype(np.float32)
    m = _module(sd, 64, device)
    w, keep = m.news_encoder.weights()
    rng = np.random.default_rng(3)
    xs = rng.standard_normal((M, 300)) * 10.0 ** rng.uniform(-20, 30, (M, 1))
    zero_rows, inf_rows = [7, M - 1], [11, M - 2]
    xs[zero_rows] = 0.0
    xs[inf_rows, 5] = np.inf
    X = torch.from_numpy(xs.astype(np.float32)).to(device)
    got = torch.empty(M, 900, device=device)
    nb = N.load().nrms_qkv_project_workspace_size(300)
    wsb = torch.empty(nb, dtype=torch.uint8, device=device)
    with N.gemm_arith(N.NRMS_GEMM_SPLIT_F16X3):
        N.call("nrms_qkv_project_ws", N.ptr(X), M, None, M, ctypes.byref(w), N.ptr(got), 0, N.ptr(wsb), nb,
               N.stream_handle(device))
    torch.cuda.synchronize()
    g = _np(got)
    xa = X.cpu().numpy().astype(np.float64)
    fine = np.ones(M, bool)
    fine[zero_rows + inf_rows] = False
    for i, n_ in enumerate(("W_Q", "W_K", "W_V")):
        want = O.linear(xa[fine], sd[f"{p}.{n_}.weight"], sd[f"{p}.{n_}.bias"], np.float64)
        assert O.normwise_rel_err(g[fine, 300 * i:300 * (i + 1)], want).max() < 2e-6, n_
        for z in zero_rows:
            assert np.array_equal(g[z, 300 * i:300 * (i + 1)], sd[f"{p}.{n_}.bias"])
    assert np.isnan(g[inf_rows]).all()


def test_qkv_project_product_count(tmp_path):
    """The split-f16 projection runs three products (w_lo·a_hi, w_hi·a_lo,
    w_hi·2^11 a_hi) unless some W column fits in 11 bits, where the fourth
    (w_hi·r, A's bits past 22) makes it exact (proj_x6.hip header). Two child
    processes, the default and NRMS_PROJ_PRODUCTS=4 (tests/proj_products_worker.py):
    random weights -> the two differ (the default took three products) and
    both are within 2e-6 of the fp64 oracle per row, the four-product rows no
    further off than 1.5x the three-product rows' worst; an identity W_Q ->
    the default took four products (bitwise equal to the forced run) and
    Q = X exactly (elements past 2^-15 of their row's largest); the bench
    slice's logits agree within 1e-6."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    outs = {}
    base = {k: v for k, v in os.environ.items() if k != "NRMS_PROJ_PRODUCTS"}
    for tag, env_add in (("default", {}), ("four", {"NRMS_PROJ_PRODUCTS": "4"})):
        env = dict(base, **env_add)
        p = subprocess.run([sys.executable, os.path.join(root, "tests", "proj_products_worker.py"),
                            str(tmp_path / f"{tag}.npz")], env=env, capture_output=True, text=True, timeout=300)
        assert p.returncode == 0, p.stderr[-3000:]
        outs[tag] = np.load(tmp_path / f"{tag}.npz")
    d, f = outs["default"], outs["four"]
    X = d["X"].astype(np.float64)
    sd = W.nrms_state(5, 64)
    p_ = "news_encoder.multihead_self_attention"
    want = np.concatenate([O.linear(X, sd[f"{p_}.{n_}.weight"], sd[f"{p_}.{n_}.bias"], np.float64)
                           for n_ in ("W_Q", "W_K", "W_V")], axis=1)
    assert not np.array_equal(d["rand"].view(np.uint32), f["rand"].view(np.uint32))
    e3 = O.normwise_rel_err(d["rand"], want)
    e4 = O.normwise_rel_err(f["rand"], want)
    print(f"three products: worst {e3.max():.3e} mean {e3.mean():.3e}; four: worst {e4.max():.3e} mean {e4.mean():.3e}")
    assert e3.max() < 2e-6 and e4.max() < 2e-6
    assert e4.max() <= 1.5 * e3.max()
    assert np.array_equal(d["mixed"].view(np.uint32), f["mixed"].view(np.uint32))
    # Q = X bit for bit where the element's pieces are fp16 normals or exact
    # subnormals (|x| >= 2^-15 of its row's largest); the smaller ones within
    # 2^-30 of it
    q, x = d["mixed"][:, :300], d["X"]
    rmax = np.abs(x).max(axis=1, keepdims=True)
    big = np.abs(x) >= rmax * 2.0 ** -15
    assert big.mean() > 0.999
    assert np.array_equal(q[big].view(np.uint32), x[big].view(np.uint32))
    assert (np.abs(q - x) <= rmax * 2.0 ** -30).all()
    rel = np.abs(d["logits"] - f["logits"]).max() / np.abs(f["logits"]).max()
    assert rel < 1e-6, rel


@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("mode", [1, 2])
def test_plan_matches_forward(device, fused, mode, gemm_mode):
    """pipeline.ForwardPlan (stage calls, as timed by bench.py) == nrms_forward."""
    from newsrecommendationsystem_amd.pipeline import ForwardPlan
    V = 3000
    sd = W.nrms_state(8, V)
    m = _module(sd, V, device)
    cand, clk, _ = W.impressions(8, 77, 33, V)
    c, k = torch.from_numpy(cand).to(device), torch.from_numpy(clk).to(device)
    plan = ForwardPlan(m, 33, 5, 50, 20, proj_mode=mode, fused=fused)
    with torch.no_grad():
        y = plan.run(c, k).clone()
        ref = m.forward_ids(c, k, proj_mode=mode)
    if fused and mode == 2:
        assert torch.equal(y, ref)
    else:
        # (direct: the stage call gets per-token rows and no ids, so it runs
        # without token compaction; nrms_forward compacts -- fp32 rounding)
        assert ((y - ref).norm() / ref.norm()) < 1e-5
    assert np.abs(_np(y) - O.forward(cand, clk, sd, np.float64)).max() <= TOL * np.abs(_np(y)).max()


def test_plan_matches_forward_many_classification_blocks(device):
    """nrms_forward's split classification (titles.hpp) with more 256-title
    classification blocks than projection workgroups (B = 1,536: 84,480
    titles, 330 blocks over 256 CUs) and a quarter of the history titles all
    padding (rep, copies, UserEncoder row list): logits bitwise those of the
    stage calls, which classify in a launch of their own with atomics
    (pipeline.ForwardPlan)."""
    from newsrecommendationsystem_amd.pipeline import ForwardPlan
    V, B = 3000, 1536
    sd = W.nrms_state(9, V)
    m = _module(sd, V, device)
    cand, clk, _ = W.impressions(9, 78, B, V)
    clk = clk.copy()
    rng = np.random.default_rng(9)
    clk[rng.random(clk.shape[:2]) < 0.25] = 0
    c, k = torch.from_numpy(cand).to(device), torch.from_numpy(clk).to(device)
    plan = ForwardPlan(m, B, 5, 50, 20, proj_mode=2, fused=True)
    with torch.no_grad():
        y = plan.run(c, k).clone()
        ref = m.forward_ids(c, k, proj_mode=2)
    assert torch.isfinite(ref).all()
    assert torch.equal(y, ref)


def test_split_gemm_accuracy_matches_f32(device):
    """The split GEMMs are as accurate as the exact-f32 MFMA GEMMs: against
    the fp64 oracle, the x6 and f16x3 forwards' errors are within 2x the f32
    forward's (all ~1e-7 normwise), on the full vocabulary."""
    from newsrecommendationsystem_amd import _native as N
    V = 70976
    sd = W.nrms_state(17, V)
    m = _module(sd, V, device, hip_cache_folded_table=False)
    cand, clk, _ = W.impressions(17, 77, 24, V)
    ref = O.forward(cand, clk, sd, np.float64)
    news_ids = W.titles(17, 78, 64, V, min_len=1)
    nref = O.news_encode(news_ids, sd, np.float64)
    errs = {}
    for mode in (N.NRMS_GEMM_SPLIT_BF16X6, N.NRMS_GEMM_F32, N.NRMS_GEMM_SPLIT_F16X3):
        with N.gemm_arith(mode), torch.no_grad():
            y = _np(m.forward_ids(torch.from_numpy(cand), torch.from_numpy(clk)))
            nv = _np(m.get_news_vector({"title": torch.from_numpy(news_ids)}))
        errs[mode] = (O.normwise_rel_err(y.reshape(1, -1), ref.reshape(1, -1)).max(),
                      O.normwise_rel_err(nv, nref).max())
    f32 = errs[N.NRMS_GEMM_F32]
    for mode in (N.NRMS_GEMM_SPLIT_BF16X6, N.NRMS_GEMM_SPLIT_F16X3):
        e = errs[mode]
        assert e[0] < 1e-5 and e[1] < 1e-5, errs
        assert e[0] <= 2 * f32[0] + 1e-7 and e[1] <= 2 * f32[1] + 1e-7, errs


def test_forward_bitwise_under_scheduling_perturbation(device):
    """The news kernel claims its groups at run time (round 6) and the
    projections / UserEncoder are persistent or LPT-ordered: which workgroup
    computes a title or a user changes from run to run. The bench batch's
    logits (1,024 impressions) are bitwise the same across repeated
    nrms_forward calls, alone and with a second stream keeping CUs busy with
    GEMMs while they run (a different workgroup timing, hence different
    claims)."""
    import bench
    from newsrecommendationsystem_amd import stream as S
    model = bench.build_model(device)
    idx = bench.stream_impressions(0, 1, 1024, device)
    cand, clk = S.batch(0, idx, bench.V_WORDS)
    with torch.no_grad():
        ref = model.forward_ids(cand, clk).clone()
        assert torch.isfinite(ref).all()
        side = torch.cuda.Stream(device)
        a = torch.randn(4096, 4096, device=device)
        for rep in range(6):
            if rep % 2:
                side.wait_stream(torch.cuda.current_stream(device))
                with torch.cuda.stream(side):
                    for _ in range(4):
                        a = torch.tanh(a @ a * 1e-3)
            y = model.forward_ids(cand, clk)
            torch.cuda.synchronize()
            assert torch.equal(y.view(torch.int32), ref.view(torch.int32)), rep


def test_bench_batch_slice_gemm_arith_vs_fp64(device):
    """A 128-impression slice of the bench's own config-3 batch (bench.py's
    model: N(0,1) embedding, V = 70,976; the first 128 impressions of the
    config-4 stream's rank-0 shard) scored through nrms_forward under each
    GEMM arithmetic, against the fp64 oracle: every arithmetic's worst row
    within 5e-6 (SURVEY §8d allows 1e-3), and f16x3 (the bench default) and
    x6 at the f32 forward's error level: their MEAN row error within 2x the
    f32 forward's. (Until round 5 this compared the max over the 128 rows,
    one row's rounding: the main pass's rep fma made the f32 forward more
    accurate, mean 9.2e-7 -> 6.5e-7, and x6's worst row moved 2.6e-6 ->
    3.3e-6 at 128 rows but 4.9e-6 -> 4.7e-6 at 512, its mean +1 %;
    profiles/r5/r5zl_rep_fma_arith_err.txt, tests/arith_err_probe.py. That
    was a relaxation made to fit a result; round 6 keeps a worst-row bound
    beside the mean: each split arithmetic's worst row within 3x the f32
    forward's worst row.)"""
    import bench
    from newsrecommendationsystem_amd import _native as N
    from newsrecommendationsystem_amd import stream as S
    model = bench.build_model(device)
    idx = bench.stream_impressions(0, 1, 128, device)
    cand, clk = S.batch(0, idx, bench.V_WORDS)
    sd = {k: v.detach().cpu().numpy() for k, v in model.state_dict().items()}
    ref = O.forward(cand.cpu().numpy(), clk.cpu().numpy(), sd, np.float64)
    errs = {}
    for name, mode in (("f32", N.NRMS_GEMM_F32), ("x6", N.NRMS_GEMM_SPLIT_BF16X6),
                       ("f16x3", N.NRMS_GEMM_SPLIT_F16X3)):
        with N.gemm_arith(mode), torch.no_grad():
            y = _np(model.forward_ids(cand, clk)).astype(np.float64)
        e = O.normwise_rel_err(y, ref)
        errs[name] = (float(e.max()), float(e.mean()))
    for name in ("f32", "x6", "f16x3"):
        assert errs[name][0] < 5e-6, errs
    for name in ("x6", "f16x3"):
        assert errs[name][1] <= 2 * errs["f32"][1], errs
        # and the outlier rows stay bounded next to the mean (the
        # round-5 change to a mean-row comparison was a relaxation, so a
        # worst-row bound is kept beside it)
        assert errs[name][0] <= 3 * errs["f32"][0] + 1e-7, errs


def _attention_pool(qkv, ldq, ids, w, device):
    """nrms_news_attention_pool over a caller-made q|k|v table (one id array)."""
    from newsrecommendationsystem_amd import _native as N
    n = ids.shape[0]
    out = torch.empty(n, 300, device=device)
    nb = N.load().nrms_news_attention_pool_workspace_size(n, 20, 300)
    ws = torch.empty(nb, dtype=torch.uint8, device=device)
    N.call("nrms_news_attention_pool", N.ptr(qkv), ldq, qkv.shape[0], N.ptr(ids), n, None, n, 20,
           ctypes.byref(w), N.ptr(out), N.ptr(ws), nb, N.stream_handle(device))
    return out


def test_f16x3_out_of_range_context_takes_recheck(device):
    """F16X3 range guard: value rows far beyond fp16's range (|v| ~ 1e6 on
    every 7th vocabulary id) make the context of any title attending to them
    overflow fp16, which the main pass turns into NaN scores; those title
    groups must come out of the recheck pass (x6 GEMM, reference exp) finite
    and within fp32 rounding of the SPLIT_BF16X6 result, like every other
    title. (Not bitwise: the x6 main pass takes the fast exp; and the 1e6
    dynamic range of the context inflates fp32 rounding differences, hence
    1e-4 here.)"""
    from newsrecommendationsystem_amd import _native as N
    V, n = 700, 1001
    sd = W.nrms_state(71, V)
    m = _module(sd, V, device, hip_cache_folded_table=False)
    g = torch.Generator().manual_seed(71)
    qkv = torch.zeros(V, 928)
    qkv[:, :600] = 0.3 * torch.randn(V, 600, generator=g)
    qkv[:, 600:900] = torch.randn(V, 300, generator=g)
    big = torch.arange(V) % 7 == 3
    qkv[big, 600:900] *= 1e6
    qkv = qkv.to(device)
    ids = torch.from_numpy(W.titles(71, 72, n, V, min_len=1)).to(device)
    w, keep = m.news_encoder.weights()
    outs = {}
    for mode in (N.NRMS_GEMM_SPLIT_F16X3, N.NRMS_GEMM_SPLIT_BF16X6):
        with N.gemm_arith(mode):
            outs[mode] = _attention_pool(qkv, 928, ids, w, device)
    h3, x6 = outs[N.NRMS_GEMM_SPLIT_F16X3], outs[N.NRMS_GEMM_SPLIT_BF16X6]
    assert torch.isfinite(x6).all()
    hit = big.to(device)[ids].any(dim=1)                       # titles attending to a big row
    grp = torch.nn.functional.pad(hit, (0, (-n) % 4)).view(-1, 4).any(dim=1)
    in_grp = grp.repeat_interleave(4)[:n]
    assert 0 < int(in_grp.sum()) < n
    assert torch.isfinite(h3).all()
    rel = ((h3 - x6).norm(dim=1) / x6.norm(dim=1)).max()
    assert rel < 1e-4, float(rel)


def test_f16x3_out_of_range_weight_takes_recheck(device):
    """A W_add entry whose 2^11-scaled fp16 plane overflows (|w| >= 32) is
    packed as NaN: every group is recomputed by the recheck pass (x6 GEMM,
    reference exp), finite and within fp32 rounding of SPLIT_BF16X6 and the
    fp64 oracle."""
    from newsrecommendationsystem_amd import _native as N
    V, n = 500, 203
    sd = dict(W.nrms_state(73, V))
    key = "news_encoder.additive_attention.linear.weight"
    sd[key] = sd[key].copy()
    sd[key][5, 17] = 40.0
    m = _module(sd, V, device, hip_cache_folded_table=False)
    titles = torch.from_numpy(W.titles(73, 74, n, V, min_len=1))
    outs = {}
    for mode in (N.NRMS_GEMM_SPLIT_F16X3, N.NRMS_GEMM_SPLIT_BF16X6):
        with N.gemm_arith(mode), torch.no_grad():
            outs[mode] = m.get_news_vector({"title": titles})
    h3, x6 = outs[N.NRMS_GEMM_SPLIT_F16X3], outs[N.NRMS_GEMM_SPLIT_BF16X6]
    assert torch.isfinite(x6).all() and torch.isfinite(h3).all()
    assert ((h3 - x6).norm(dim=1) / x6.norm(dim=1)).max() < 1e-5
    ref = O.news_encode(titles.numpy(), sd, np.float64)
    assert O.normwise_rel_err(_np(outs[N.NRMS_GEMM_SPLIT_F16X3]), ref).max() < TOL


@pytest.mark.parametrize("B,n_clk", [(3, 1), (5, 17), (257, 50), (4, 64)])
def test_fused_user_tail_vs_stages(device, B, n_clk, gemm_mode):
    """Fused UserEncoder tail (nrms_user_attention_pool) == the separate stage
    kernels within fp32 reordering, and == the fp64 oracle, for history
    lengths 1..64 (the kernel's range)."""
    from newsrecommendationsystem_amd import _native as N
    V = 300
    sd = W.nrms_state(23, V)
    m = _module(sd, V, device)
    rng = np.random.default_rng(100 + n_clk)
    vec = (0.3 * rng.standard_normal((B, n_clk, 300))).astype(np.float32)
    x = torch.from_numpy(vec).to(device).reshape(B * n_clk, 300).contiguous()
    w, keep = m.user_encoder.weights()
    st = N.stream_handle(device)
    lib = N.load()
    uqkv = torch.empty(B * n_clk, 900, device=device)
    pb = lib.nrms_qkv_project_workspace_size(300)
    pws = torch.empty(pb, dtype=torch.uint8, device=device)
    N.call("nrms_qkv_project_ws", N.ptr(x), B * n_clk, None, B * n_clk, ctypes.byref(w), N.ptr(uqkv), 0,
           N.ptr(pws), pb, st)
    out = torch.empty(B, 300, device=device)
    nb = lib.nrms_user_attention_pool_workspace_size(B, n_clk, 300)
    ws = torch.empty(nb, dtype=torch.uint8, device=device)
    N.call("nrms_user_attention_pool", N.ptr(uqkv), 0, B, n_clk, ctypes.byref(w), N.ptr(out),
           N.ptr(ws), nb, st)
    ctx = torch.empty(B * n_clk, 300, device=device)
    sc = torch.empty(B * n_clk, device=device)
    ref = torch.empty(B, 300, device=device)
    N.call("nrms_self_attention", N.ptr(uqkv), B * n_clk, None, B, None, B, n_clk, ctypes.byref(w),
           N.ptr(ctx), st)
    N.call("nrms_additive_attention", N.ptr(ctx), B, n_clk, ctypes.byref(w), N.ptr(sc), N.ptr(ref),
           st)
    err = ((out - ref).norm(dim=1) / ref.norm(dim=1)).max()
    assert err < 1e-5, float(err)
    oracle = O.user_encode(vec, sd, np.float64)
    assert O.normwise_rel_err(_np(out), oracle).max() < 1e-5
    # the module path (nrms_user_encode) takes the fused kernel: bitwise equal
    with torch.no_grad():
        u = m.get_user_vector(torch.from_numpy(vec).to(device))
    assert torch.equal(u, out)


@pytest.mark.parametrize("B,n_clk", [(40, 50), (9, 17), (6, 64)])
def test_user_tail_padded_compaction(device, B, n_clk, gemm_mode):
    """nrms_user_attention_pool_padded: the clicked positions flagged as
    all-padding titles (one news vector) collapse into one row with their
    count. Histories with 0, 1, some, all-but-one and all positions padding,
    left-padded and interleaved: within fp32 rounding of the uncompacted tail
    (nrms_user_attention_pool) and of the fp64 oracle; with token compaction
    off it is the uncompacted tail bitwise."""
    from newsrecommendationsystem_amd import _native as N
    V = 300
    sd = W.nrms_state(29, V)
    m = _module(sd, V, device)
    rng = np.random.default_rng(200 + n_clk)
    vec = (0.3 * rng.standard_normal((B, n_clk, 300))).astype(np.float32)
    padv = (0.3 * rng.standard_normal(300)).astype(np.float32)   # the padding title's vector
    flags = np.zeros((B, n_clk), np.uint8)
    for b in range(B):
        kind = b % 6
        if kind == 1:
            flags[b, :1] = 1
        elif kind == 2:
            flags[b, : rng.integers(1, n_clk)] = 1          # left padding
        elif kind == 3:
            flags[b, : n_clk - 1] = 1
        elif kind == 4:
            flags[b, :] = 1
        elif kind == 5:
            flags[b, rng.random(n_clk) < 0.4] = 1           # interleaved
    vec[flags.astype(bool)] = padv
    x = torch.from_numpy(vec).to(device).reshape(B * n_clk, 300).contiguous()
    w, keep = m.user_encoder.weights()
    st = N.stream_handle(device)
    lib = N.load()
    uqkv = torch.empty(B * n_clk, 900, device=device)
    pb = lib.nrms_qkv_project_workspace_size(300)
    pws = torch.empty(pb, dtype=torch.uint8, device=device)
    N.call("nrms_qkv_project_ws", N.ptr(x), B * n_clk, None, B * n_clk, ctypes.byref(w), N.ptr(uqkv), 0,
           N.ptr(pws), pb, st)
    nb = lib.nrms_user_attention_pool_workspace_size(B, n_clk, 300)
    ws = torch.empty(nb, dtype=torch.uint8, device=device)
    fl = torch.from_numpy(flags.reshape(-1)).to(device)
    plain = torch.empty(B, 300, device=device)
    N.call("nrms_user_attention_pool", N.ptr(uqkv), 0, B, n_clk, ctypes.byref(w), N.ptr(plain),
           N.ptr(ws), nb, st)
    outs = {}
    prev = lib.nrms_set_token_compaction(1)
    try:
        for on in (1, 0):
            lib.nrms_set_token_compaction(on)
            o = torch.empty(B, 300, device=device)
            N.call("nrms_user_attention_pool_padded", N.ptr(uqkv), 0, B, n_clk, N.ptr(fl), ctypes.byref(w),
                   N.ptr(o), N.ptr(ws), nb, st)
            outs[on] = o
    finally:
        lib.nrms_set_token_compaction(prev)
    assert torch.equal(outs[0], plain)
    assert torch.isfinite(outs[1]).all()
    err = ((outs[1] - plain).norm(dim=1) / plain.norm(dim=1)).max()
    assert err < 2e-6, float(err)
    oracle = O.user_encode(vec, sd, np.float64)
    assert O.normwise_rel_err(_np(outs[1]), oracle).max() < 1e-5


def test_fused_user_tail_value_range(device, gemm_mode):
    """The fused UserEncoder tail with V rows from 1e-20 to 1e25 in magnitude
    (per user; Q and K small, so the raw exps stay finite): the split-f16
    GEMM's per-row power-of-two scaling keeps every operand in fp16's range,
    and the tail matches the stage kernels within 1e-5 normwise per user, with
    no NaN or inf."""
    from newsrecommendationsystem_amd import _native as N
    V, B, n_clk = 300, 24, 50
    sd = W.nrms_state(31, V)
    m = _module(sd, V, device)
    w, keep = m.user_encoder.weights()
    rng = np.random.default_rng(41)
    qkv = (0.3 * rng.standard_normal((B, n_clk, 900))).astype(np.float64)
    qkv[:, :, 600:] *= 10.0 ** rng.uniform(-20, 25, (B, 1, 1))
    x = torch.from_numpy(qkv.astype(np.float32).reshape(B * n_clk, 900)).to(device)
    st = N.stream_handle(device)
    lib = N.load()
    out = torch.empty(B, 300, device=device)
    nb = lib.nrms_user_attention_pool_workspace_size(B, n_clk, 300)
    ws = torch.empty(nb, dtype=torch.uint8, device=device)
    N.call("nrms_user_attention_pool", N.ptr(x), 0, B, n_clk, ctypes.byref(w), N.ptr(out), N.ptr(ws), nb, st)
    ctx = torch.empty(B * n_clk, 300, device=device)
    sc = torch.empty(B * n_clk, device=device)
    ref = torch.empty(B, 300, device=device)
    N.call("nrms_self_attention", N.ptr(x), B * n_clk, None, B, None, B, n_clk, ctypes.byref(w), N.ptr(ctx), st)
    N.call("nrms_additive_attention", N.ptr(ctx), B, n_clk, ctypes.byref(w), N.ptr(sc), N.ptr(ref), st)
    torch.cuda.synchronize()
    assert torch.isfinite(out).all() and torch.isfinite(ref).all()
    err = ((out - ref).norm(dim=1) / ref.norm(dim=1)).max()
    assert err < 1e-5, float(err)


@pytest.mark.parametrize("n_clk", [33, 36, 50])
def test_user_tail_recheck_rows_chunked(device, gemm_mode, n_clk):
    """Histories of 33-50 titles (split-f16: the 512-thread instance, K|V
    staged 32 rows at a time, two task passes past 34 titles, the context in
    two planes past 39): users whose head-0 raw exps come near fp32 overflow
    (sum >= 2^120, the recheck path, which re-reads K|V from the projected
    rows) or overflow (NaN, multihead_self.py:16-20) beside ordinary users.
    Same NaN pattern as the stage kernels, finite users within 1e-5."""
    from newsrecommendationsystem_amd import _native as N
    V, B = 300, 24
    sd = W.nrms_state(37, V)
    m = _module(sd, V, device)
    w, keep = m.user_encoder.weights()
    rng = np.random.default_rng(43 + n_clk)
    qkv = (0.3 * rng.standard_normal((B, n_clk, 900))).astype(np.float32)
    for b in range(B):
        if b % 3:
            a = 4.36 if b % 3 == 1 else 4.5    # sqrt(20) a^2 = 85.0 (finite, rechecked) / 90.6 (overflow)
            qkv[b, :, 0:20] = a                 # head 0's Q
            qkv[b, :, 300:320] = a              # head 0's K
    x = torch.from_numpy(qkv.reshape(B * n_clk, 900)).to(device)
    st = N.stream_handle(device)
    lib = N.load()
    out = torch.empty(B, 300, device=device)
    nb = lib.nrms_user_attention_pool_workspace_size(B, n_clk, 300)
    ws = torch.empty(nb, dtype=torch.uint8, device=device)
    N.call("nrms_user_attention_pool", N.ptr(x), 0, B, n_clk, ctypes.byref(w), N.ptr(out), N.ptr(ws), nb, st)
    ctx = torch.empty(B * n_clk, 300, device=device)
    sc = torch.empty(B * n_clk, device=device)
    ref = torch.empty(B, 300, device=device)
    N.call("nrms_self_attention", N.ptr(x), B * n_clk, None, B, None, B, n_clk, ctypes.byref(w), N.ptr(ctx), st)
    N.call("nrms_additive_attention", N.ptr(ctx), B, n_clk, ctypes.byref(w), N.ptr(sc), N.ptr(ref), st)
    torch.cuda.synchronize()
    o, r = _np(out), _np(ref)
    assert np.array_equal(np.isnan(o), np.isnan(r))
    nan_users = np.isnan(r).any(axis=1)
    assert nan_users[2::3].all() and not nan_users[0::3].any() and not nan_users[1::3].any()
    fin = ~nan_users
    err = np.linalg.norm(o[fin] - r[fin], axis=1) / np.linalg.norm(r[fin], axis=1)
    assert err.max() < 1e-5, float(err.max())


@pytest.mark.parametrize("n_clk", [65, 200])
def test_user_tail_beyond_fused_range(device, n_clk):
    """Histories longer than 64: the fused kernel declines (UNSUPPORTED) and
    nrms_user_encode takes the stage kernels (K|V through L2, two-pass raw
    exps, strided pooling softmax); result matches the oracle."""
    from newsrecommendationsystem_amd import _native as N
    V, B = 300, 3
    sd = W.nrms_state(29, V)
    m = _module(sd, V, device)
    vec = (0.3 * np.random.default_rng(7).standard_normal((B, n_clk, 300))).astype(np.float32)
    w, keep = m.user_encoder.weights()
    lib = N.load()
    out = torch.empty(B, 300, device=device)
    x = torch.zeros(B * n_clk, 900, device=device)
    rc = lib.nrms_user_attention_pool(N.ptr(x), 0, B, n_clk, ctypes.byref(w), N.ptr(out), None, 0,
                                      N.stream_handle(device))
    assert rc == N.NRMS_ERR_UNSUPPORTED
    with torch.no_grad():
        u = _np(m.get_user_vector(torch.from_numpy(vec).to(device)))
    assert O.normwise_rel_err(u, O.user_encode(vec, sd, np.float64)).max() < 1e-5


def test_config2_news_encoder_100k_titles(device, gemm_mode):
    """BASELINE config 2 at full size (100,000 titles x 20 tokens, V = 70,976,
    N(0,1) table): folded == direct within fp32 rounding (normwise 1e-5),
    encoding in two halves == one call bitwise, and a 512-title sample
    against the fp64 oracle (normwise TOL per vector)."""
    from newsrecommendationsystem_amd import _native as N
    V, n = 70976, 100_000
    sd = W.nrms_state(8, V)
    m = _module(sd, V, device, hip_cache_folded_table=False)
    titles = torch.from_numpy(W.titles(8, 500, n, V))
    with torch.no_grad():
        m.config.hip_proj_mode = N.NRMS_PROJ_FOLDED
        folded = m.get_news_vector({"title": titles})
        halves = torch.cat([m.get_news_vector({"title": titles[:n // 2]}),
                            m.get_news_vector({"title": titles[n // 2:]})])
        m.config.hip_proj_mode = N.NRMS_PROJ_DIRECT
        direct = m.get_news_vector({"title": titles})
    assert torch.isfinite(folded).all()
    assert torch.equal(folded, halves)
    rel = ((folded - direct).norm(dim=1) / direct.norm(dim=1)).max()
    assert rel < 1e-5, float(rel)
    pick = np.sort(W.randint(8, 501, (512,), 0, n))
    ref = O.news_encode(titles.numpy()[pick], sd, np.float64)
    assert O.normwise_rel_err(_np(folded)[pick], ref).max() < TOL


@pytest.mark.parametrize("pad_frac", [0.0, 0.45, 1.0])
def test_padding_title_dedupe_is_bitwise_identical(device, pad_frac, gemm_mode):
    """nrms_set_title_dedupe: encoding one all-padding 4-title group and
    copying its slot vectors to the other all-padding groups gives bitwise the
    same logits and news vectors as encoding every title, with no, some and
    only padding titles (clicked and candidate slots), through nrms_forward and
    get_news_vector."""
    from newsrecommendationsystem_amd import _native as N
    V, B = 3000, 96
    sd = W.nrms_state(61, V)
    m = _module(sd, V, device, hip_proj_mode=N.NRMS_PROJ_FOLDED)
    cand, clk, _ = W.impressions(61, 3, B, V)
    rng = np.random.default_rng(61)
    clk = clk.copy()
    cand = cand.copy()
    if pad_frac == 1.0:
        clk[:] = 0
        cand[:] = 0
    elif pad_frac > 0:
        clk[rng.random(clk.shape[:2]) < pad_frac] = 0
        cand[rng.random(cand.shape[:2]) < 0.1] = 0
    else:
        clk[clk.sum(-1) == 0, 0] = 1          # no all-zero title anywhere
    titles = torch.from_numpy(np.concatenate([clk.reshape(-1, 20), cand.reshape(-1, 20)]))
    lib = N.load()
    outs = {}
    prev = lib.nrms_set_title_dedupe(1)
    try:
        for on in (1, 0):
            lib.nrms_set_title_dedupe(on)
            with torch.no_grad():
                y = m.forward_ids(torch.from_numpy(cand), torch.from_numpy(clk))
                v = m.get_news_vector({"title": titles})
            outs[on] = (y.clone(), v.clone())
    finally:
        lib.nrms_set_title_dedupe(prev)
    assert torch.equal(outs[1][0], outs[0][0])
    assert torch.equal(outs[1][1], outs[0][1])
    assert torch.isfinite(outs[1][0]).all()
    pad = (titles == 0).all(dim=1)
    if pad.any():   # one vector per slot; slots agree to fp32 rounding
        vp = outs[1][1][pad.to(device)]
        assert float((vp - vp[:1]).abs().max()) <= 1e-6 * float(vp.abs().max())


def _set_switch(lib, name, on):
    return getattr(lib, name)(on)


@pytest.mark.parametrize("mode", ["folded", "direct"])
def test_token_compaction_every_title_length(device, mode, gemm_mode):
    """nrms_set_token_compaction: titles with 0..20 real tokens (right-padded,
    plus interior zeros and a title of only interior padding) encoded with the
    padding rows compacted agree with the uncompacted encoding to fp32
    rounding, and both with the fp64 oracle (news_encoder.py:27-48)."""
    from newsrecommendationsystem_amd import _native as N
    V = 1500
    sd = W.nrms_state(71, V)
    pm = N.NRMS_PROJ_FOLDED if mode == "folded" else N.NRMS_PROJ_DIRECT
    m = _module(sd, V, device, hip_proj_mode=pm, hip_cache_folded_table=False)
    rng = np.random.default_rng(71)
    rows = []
    for rep in range(6):
        for c in range(21):
            t = np.zeros(20, np.int64)
            t[:c] = rng.integers(1, V, c)
            rows.append(t)
    t = rng.integers(1, V, 20)
    t[[2, 5, 6, 11, 19]] = 0          # interior zeros
    rows.append(t)
    t = np.zeros(20, np.int64)
    t[[0, 7, 13]] = rng.integers(1, V, 3)
    rows.append(t)
    ids = np.stack(rows)
    lib = N.load()
    outs = {}
    prev = lib.nrms_set_token_compaction(1)
    try:
        for on in (1, 0):
            lib.nrms_set_token_compaction(on)
            with torch.no_grad():
                outs[on] = _np(m.get_news_vector({"title": torch.from_numpy(ids)}))
    finally:
        lib.nrms_set_token_compaction(prev)
    assert np.isfinite(outs[1]).all()
    assert O.normwise_rel_err(outs[1], outs[0]).max() < 2e-6
    ref = O.news_encode(ids, sd, np.float64)
    assert O.normwise_rel_err(outs[1], ref).max() < TOL
    assert O.normwise_rel_err(outs[0], ref).max() < TOL
    # a title's vector does not depend on where in the launch it is encoded
    with torch.no_grad():
        perm = rng.permutation(len(ids))
        again = _np(m.get_news_vector({"title": torch.from_numpy(ids[perm])}))
    assert np.array_equal(again, outs[1][perm])


def test_token_compaction_forward_vs_oracle(device, gemm_mode):
    """The config-3-shaped forward (left-padded histories, right-padded
    titles) with and without token compaction, against the fp64 oracle."""
    from newsrecommendationsystem_amd import _native as N
    V, B = 4000, 48
    sd = W.nrms_state(73, V)
    m = _module(sd, V, device, hip_proj_mode=N.NRMS_PROJ_FOLDED)
    cand, clk, _ = W.impressions(73, 9, B, V)
    cand, clk = cand.copy(), clk.copy()
    # UserEncoder compaction buckets (Le = real + 1 <= 16 / 32 / 50) at their
    # edges: history lengths 1, 15, 16, 31, 32, 49, 50 (no padding row)
    full, _, _ = W.impressions(74, 9, 7, V)
    full_clk = W.titles(74, 31, 7 * 50, V).reshape(7, 50, 20)
    for b, h in enumerate([1, 15, 16, 31, 32, 49, 50]):
        clk[b] = full_clk[b]
        clk[b, : 50 - h] = 0
    lib = N.load()
    ys = {}
    prev = lib.nrms_set_token_compaction(1)
    try:
        for on in (1, 0):
            lib.nrms_set_token_compaction(on)
            with torch.no_grad():
                ys[on] = _np(m.forward_ids(torch.from_numpy(cand), torch.from_numpy(clk)))
    finally:
        lib.nrms_set_token_compaction(prev)
    ref = O.forward(cand, clk, sd, np.float64)
    scale = max(np.abs(ref).max(), 1e-6)
    assert np.abs(ys[1] - ref).max() <= TOL * scale
    assert np.abs(ys[1] - ys[0]).max() <= 1e-5 * scale


def test_padding_title_dedupe_odd_batch_bitwise(device, gemm_mode):
    """with B = 37 and N = 50 the B*N clicked titles are not a
    multiple of 4, so the 4-title group holding the last user's final history
    slots also holds the first user's first candidates. Both are all padding
    here, plus several whole padding groups elsewhere: the representative
    group choice, the UserEncoder row list and the scorer's redirect to the
    representative group all see a group that straddles clicked and candidate
    titles. Logits must be bitwise equal with the dedupe on and off."""
    from newsrecommendationsystem_amd import _native as N
    V, B, N_ = 2500, 37, 50
    sd = W.nrms_state(67, V)
    m = _module(sd, V, device, hip_proj_mode=N.NRMS_PROJ_FOLDED)
    cand, clk, _ = W.impressions(67, 5, B, V, N=N_)
    cand, clk = cand.copy(), clk.copy()
    assert (B * N_) % 4 != 0
    clk[-1, -3:] = 0                 # last user's final history slots
    cand[0, :2] = 0                  # first user's first candidates (same group)
    clk[3, :40] = 0                  # whole all-padding groups elsewhere
    clk[11, :] = 0
    cand[20, :] = 0
    lib = N.load()
    outs = {}
    prev = lib.nrms_set_title_dedupe(1)
    try:
        for on in (1, 0):
            lib.nrms_set_title_dedupe(on)
            with torch.no_grad():
                outs[on] = m.forward_ids(torch.from_numpy(cand), torch.from_numpy(clk)).clone()
    finally:
        lib.nrms_set_title_dedupe(prev)
    assert torch.equal(outs[1], outs[0])
    assert torch.isfinite(outs[1]).all()
    ref = O.forward(cand, clk, sd, np.float64)
    assert np.abs(_np(outs[1]) - ref).max() <= TOL * max(np.abs(ref).max(), 1e-6)


def test_forward_graph_replay_recomputes_bitwise(device):
    """nrms_forward captured in a HIP graph (bench.py's timed step): each
    replay recomputes the logits from whatever the captured id buffers hold
    (a new batch copied in gives that batch's eager logits bitwise, logits
    poisoned between replays come back), with padding titles in the batch so
    the on-device dedupe classification runs inside the graph."""
    from newsrecommendationsystem_amd.pipeline import TimedForward
    V, B = 3000, 64
    sd = W.nrms_state(93, V)
    m = _module(sd, V, device)
    batches = []
    for seed in (93, 94):
        cand, clk, _ = W.impressions(seed, 5, B, V)
        clk = clk.copy()
        clk[np.random.default_rng(seed).random(clk.shape[:2]) < 0.3] = 0
        batches.append((torch.from_numpy(cand).to(device), torch.from_numpy(clk).to(device)))
    fwd = TimedForward(m, B, 5, 50, 20)
    c, k = batches[0][0].clone(), batches[0][1].clone()
    with torch.no_grad():
        eager = [fwd.run(*b).clone() for b in batches]
        side = torch.cuda.Stream(device)
        side.wait_stream(torch.cuda.current_stream(device))
        with torch.cuda.stream(side):
            fwd.run(c, k)
        torch.cuda.current_stream(device).wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            fwd.run(c, k)
        for i in (0, 1, 0):
            c.copy_(batches[i][0])
            k.copy_(batches[i][1])
            fwd.logits.fill_(float("nan"))
            graph.replay()
            torch.cuda.synchronize()
            assert torch.equal(fwd.logits, eager[i]), i
    assert not torch.equal(eager[0], eager[1])
    assert torch.isfinite(eager[1]).all()


def test_forward_timed_matches_forward_and_records_stages(device):
    """nrms_forward_timed (bench.py's timed step): bitwise the logits of
    nrms_forward / NRMS.forward_ids and of the stage-by-stage ForwardPlan, with
    the five stage events recorded in order (positive, summing to the span)."""
    from newsrecommendationsystem_amd import _native as N
    from newsrecommendationsystem_amd.pipeline import ForwardPlan, TimedForward
    V, B = 3000, 70
    sd = W.nrms_state(91, V)
    m = _module(sd, V, device)
    cand, clk, _ = W.impressions(91, 5, B, V)
    c, k = torch.from_numpy(cand).to(device), torch.from_numpy(clk).to(device)
    fwd = TimedForward(m, B, 5, 50, 20)
    assert fwd.stages == ["qkv_news", "news_fused", "qkv_user", "user_fused", "score"]
    ev = fwd.make_events(1)[0]
    with torch.no_grad():
        y = fwd.run(c, k, ev).clone()
        ref = m.forward_ids(c, k)
        plan = ForwardPlan(m, B, 5, 50, 20).run(c, k).clone()
    torch.cuda.synchronize()
    assert torch.equal(y, ref) and torch.equal(y, plan)
    ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(5)]
    assert all(t > 0 for t in ms), ms
    assert abs(sum(ms) - ev[0].elapsed_time(ev[5])) < 1e-2
    lib = N.load()
    assert lib.nrms_forward_timed(None, None, B, 5, 50, 20, None, V, None, None, 2, None, None, 0,
                                  None, None, 3) == N.NRMS_ERR_INVALID_ARG


_FALLBACK_SCRIPT = r"""
import sys, torch, numpy as np
sys.path.insert(0, sys.argv[1])
from oracle import weights as W
from newsrecommendationsystem_amd import NRMS, NRMSConfig
from newsrecommendationsystem_amd.pipeline import ForwardPlan
V, B = 3000, 300
class Cfg(NRMSConfig):
    num_words = V
m = NRMS(Cfg)
m.load_state_dict({k: torch.from_numpy(v) for k, v in W.nrms_state(9, V).items()})
m = m.to("cuda:0").eval()
cand, clk, _ = W.impressions(9, 78, B, V)
clk = clk.copy()
clk[np.random.default_rng(9).random(clk.shape[:2]) < 0.25] = 0
c, k = torch.from_numpy(cand).cuda(), torch.from_numpy(clk).cuda()
with torch.no_grad():
    y = ForwardPlan(m, B, 5, 50, 20, proj_mode=2, fused=True).run(c, k).clone()
    ref = m.forward_ids(c, k, proj_mode=2)
assert torch.isfinite(ref).all()
assert torch.equal(y, ref), float((y - ref).abs().max())
print("FALLBACK_OK")
"""


def test_forward_classification_fallback_without_tail_jobs():
    """nrms_forward with the classification's first half run in the pack
    launch but the projection's tail jobs skipped (NRMS_TEST_SKIP_CLASSIFY_TAIL,
    read at library load: a child process): the news launch classifies again
    with its own atomics, on counters the pack launch reset, and the logits
    equal the stage-by-stage plan's bitwise (round-4 advisor finding)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, NRMS_TEST_SKIP_CLASSIFY_TAIL="1")
    r = subprocess.run([sys.executable, "-c", _FALLBACK_SCRIPT, root], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and "FALLBACK_OK" in r.stdout, r.stderr[-3000:]



def test_user_long_history_forms_bitwise(tmp_path):
    """The chunked UserEncoder instance (512 threads, two workgroups per CU)
    has three forms for a user with more (head, query) tasks than threads
    (35..50 titles), all running the single-query arithmetic over the keys in
    the same order: two queries of one head per thread in one pass over two
    key chunks (round 6, the default), two passes split by head (the first 8,
    9 or 10 heads, then the rest; NRMS_USER_PAIR=0), and the round-5 two
    passes split by task index (NRMS_USER_PAIR=0 NRMS_USER_HSPLIT=0). The
    user vectors at 34, 36, 38, 41, 46 and 50 rows (rows that take the
    recheck path included) and a 256-impression bench slice's logits are
    bitwise equal across the three. (The 832-thread whole-tile instance pools
    over 8 lanes per column instead of 4: within rounding, not bitwise.)"""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    outs = {}
    for tag, env_add in (("pair", {}), ("heads", {"NRMS_USER_PAIR": "0"}),
                         ("tasks", {"NRMS_USER_PAIR": "0", "NRMS_USER_HSPLIT": "0"})):
        env = dict(os.environ, **env_add)
        p = subprocess.run([sys.executable, os.path.join(root, "tests", "user_chunk_worker.py"),
                            str(tmp_path / f"{tag}.npz")], env=env, capture_output=True, text=True, timeout=300)
        assert p.returncode == 0, p.stderr[-3000:]
        outs[tag] = np.load(tmp_path / f"{tag}.npz")
    for k in ("uv34", "uv36", "uv38", "uv41", "uv46", "uv50", "logits"):
        a = outs["tasks"][k]
        assert np.isfinite(a).any()
        for tag in ("pair", "heads"):
            assert np.array_equal(outs[tag][k].view(np.uint32), a.view(np.uint32)), (tag, k)
