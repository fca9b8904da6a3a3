"""NRMS on MI355X: the reference's module interface, computed by libnrms_hip.

Drop-in for ``model.NRMS.NRMS`` (src/model/NRMS/__init__.py:7-84): same
constructor ``NRMS(config, pretrained_word_embedding=None)``, same
``forward(candidate_news, clicked_news)``, ``get_news_vector``,
``get_user_vector`` and ``get_prediction`` signatures, and the same
sub-module / parameter names, so reference ``state_dict`` checkpoints load
unchanged (src/train.py:266-277, src/evaluate.py:281-288).

Every forward computation runs in the HIP kernels behind the C ABI
(include/nrms_hip.h); parameters are only stored here. There is no CPU or
eager fallback: without the built library every call raises.

Differences from the reference that a caller can observe:
  * the device is the module's own device (``.to(device)``), not a global
    ``cuda:0`` (src/model/NRMS/news_encoder.py:7), so one process per GPU works;
  * training mode (``model.train()``) on a GPU runs the HIP training kernels
    (train_hip.py: train-mode forward with dropout, backward through a
    torch.autograd.Function) so src/train.py can drive this module unchanged;
    on CPU (or with ``config.hip_train = False``) the reference's op sequence
    runs on ATen autograd (newsrecommendationsystem_amd/train.py). Dropout
    masks come from the library's counter-based generator, not torch's RNG.
"""
import torch
import torch.nn as nn

from . import _native as N
from . import train as _train
from .config import NRMSConfig


def _f32(t):
    if t.dtype != torch.float32 or not t.is_contiguous():
        t = t.float().contiguous()
    return t


class MultiHeadSelfAttention(nn.Module):
    """Parameter holder for src/model/general/attention/multihead_self.py:26-44."""

    def __init__(self, d_model, num_attention_heads):
        super().__init__()
        assert d_model % num_attention_heads == 0
        self.d_model = d_model
        self.num_attention_heads = num_attention_heads
        self.d_k = self.d_v = d_model // num_attention_heads
        self.W_Q = nn.Linear(d_model, d_model)
        self.W_K = nn.Linear(d_model, d_model)
        self.W_V = nn.Linear(d_model, d_model)
        for lin in (self.W_Q, self.W_K, self.W_V):
            nn.init.xavier_uniform_(lin.weight, gain=1)


class AdditiveAttention(nn.Module):
    """Parameter holder for src/model/general/attention/additive.py:6-20."""

    def __init__(self, query_vector_dim, candidate_vector_dim):
        super().__init__()
        self.linear = nn.Linear(candidate_vector_dim, query_vector_dim)
        self.attention_query_vector = nn.Parameter(torch.empty(query_vector_dim).uniform_(-0.1, 0.1))


def _encoder_struct(mhsa, add):
    """nrms_encoder_weights_t over the live parameter storage (no copies when
    the parameters are contiguous fp32, which nn.Linear's are)."""
    keep = [_f32(t.detach()) for t in (mhsa.W_Q.weight, mhsa.W_Q.bias, mhsa.W_K.weight,
                                       mhsa.W_K.bias, mhsa.W_V.weight, mhsa.W_V.bias,
                                       add.linear.weight, add.linear.bias,
                                       add.attention_query_vector)]
    s = N.EncoderWeights(*[t.data_ptr() for t in keep], mhsa.d_model, mhsa.num_attention_heads,
                         add.linear.out_features)
    return s, keep


class _Workspace:
    """Grow-only device scratch handed to the library (caller-owned memory)."""

    def __init__(self):
        self.buf = None

    def get(self, nbytes, device):
        nbytes = max(int(nbytes), 256)
        if self.buf is None or self.buf.numel() < nbytes or self.buf.device != device:
            self.buf = torch.empty(nbytes, dtype=torch.uint8, device=device)
        return self.buf


class NewsEncoder(nn.Module):
    """src/model/NRMS/news_encoder.py:10-48, forward on the HIP path."""

    def __init__(self, config, pretrained_word_embedding=None):
        super().__init__()
        self.config = config
        if pretrained_word_embedding is None:
            self.word_embedding = nn.Embedding(config.num_words, config.word_embedding_dim,
                                               padding_idx=0)
        else:
            self.word_embedding = nn.Embedding.from_pretrained(pretrained_word_embedding,
                                                               freeze=False, padding_idx=0)
        self.multihead_self_attention = MultiHeadSelfAttention(config.word_embedding_dim,
                                                               config.num_attention_heads)
        self.additive_attention = AdditiveAttention(config.query_vector_dim,
                                                    config.word_embedding_dim)
        self._ws = _Workspace()
        self._folded = None  # (key, qkv_table)

    # -- helpers --------------------------------------------------------------
    def weights(self):
        return _encoder_struct(self.multihead_self_attention, self.additive_attention)

    def table(self):
        return _f32(self.word_embedding.weight.detach())

    def _ids(self, title):
        dev = self.word_embedding.weight.device
        if getattr(self.config, "hip_check_ids", True) and title.numel():
            lo, hi = torch.aminmax(title)  # CPU input: no device sync
            V = self.word_embedding.num_embeddings
            if int(lo) < 0 or int(hi) >= V:
                raise IndexError("index out of range in self")
        return title.to(device=dev, dtype=torch.int64, non_blocking=True).contiguous()

    def _fold_key(self):
        ps = [self.word_embedding.weight] + [
            getattr(getattr(self.multihead_self_attention, n), a)
            for n in ("W_Q", "W_K", "W_V") for a in ("weight", "bias")]
        return tuple((p.data_ptr(), p._version) for p in ps) + (N.load().nrms_get_gemm_arith(),)

    def folded_table(self):
        """Projected vocabulary [V, 3D] (E [W_Q;W_K;W_V]^T + b), cached while
        the embedding and Q/K/V parameters are unchanged (tensor versions)."""
        key = self._fold_key()
        if self._folded is not None and self._folded[0] == key:
            return self._folded[1]
        tab = self.table()
        V, D = tab.shape
        w, keep = self.weights()
        ld = N.load().nrms_qkv_row_stride(D)
        qkv = torch.empty(V, ld, dtype=torch.float32, device=tab.device)
        nb = N.load().nrms_qkv_project_workspace_size(D)   # the pre-split-W projection, as nrms_forward's
        ws = torch.empty(nb, dtype=torch.uint8, device=tab.device)
        N.call("nrms_qkv_project_ws", N.ptr(tab), V, None, V, ctypes_byref(w), N.ptr(qkv), ld, N.ptr(ws), nb,
               N.stream_handle(tab.device))
        self._folded = (key, qkv)
        return qkv

    # -- reference interface --------------------------------------------------
    def forward(self, news):
        if self.training:
            return _train.news_encode_autograd(self, self._ids(news["title"]))
        ids = self._ids(news["title"])
        n, L = ids.shape
        tab = self.table()
        V, D = tab.shape
        out = torch.empty(n, D, dtype=torch.float32, device=tab.device)
        if n == 0:
            return out
        w, keep = self.weights()
        stream = N.stream_handle(tab.device)
        mode = getattr(self.config, "hip_proj_mode", N.NRMS_PROJ_AUTO)
        if getattr(self.config, "hip_cache_folded_table", True) and mode != N.NRMS_PROJ_DIRECT:
            qkv = self.folded_table()
            nb = N.load().nrms_news_encode_folded_workspace_size(n, L, D)
            ws = self._ws.get(nb, tab.device)
            N.call("nrms_news_encode_folded", N.ptr(ids), n, L, N.ptr(qkv), qkv.shape[1], V,
                   ctypes_byref(w),
                   N.ptr(out), N.ptr(ws), ws.numel(), stream)
        else:
            nb = N.load().nrms_news_encode_workspace_size(n, L, V, D, mode)
            ws = self._ws.get(nb, tab.device)
            N.call("nrms_news_encode", N.ptr(ids), n, L, N.ptr(tab), V, ctypes_byref(w), mode,
                   N.ptr(out), N.ptr(ws), ws.numel(), stream)
        return out


class UserEncoder(nn.Module):
    """src/model/NRMS/user_encoder.py:6-26, forward on the HIP path."""

    def __init__(self, config):
        super().__init__()
        self.config = config
        self.multihead_self_attention = MultiHeadSelfAttention(config.word_embedding_dim,
                                                               config.num_attention_heads)
        self.additive_attention = AdditiveAttention(config.query_vector_dim,
                                                    config.word_embedding_dim)
        self._ws = _Workspace()

    def weights(self):
        return _encoder_struct(self.multihead_self_attention, self.additive_attention)

    def forward(self, user_vector):
        if self.training:
            dev = self.additive_attention.attention_query_vector.device
            return _train.user_encode_autograd(self, user_vector.to(dev))
        dev = self.additive_attention.attention_query_vector.device
        x = user_vector.to(dev)
        B, n_clicked, D = x.shape
        # strided [B, N, D] views (the transpose(0, 1) of src/evaluate.py:220-224)
        # are read in place; only an inner stride != 1 or a misaligned view is copied
        if (x.dtype != torch.float32 or x.stride(2) != 1 or x.stride(0) % 4 or x.stride(1) % 4
                or x.data_ptr() % 16):
            x = _f32(x)
        out = torch.empty(B, D, dtype=torch.float32, device=dev)
        if B == 0:
            return out
        w, keep = self.weights()
        nb = N.load().nrms_user_encode_workspace_size(B, n_clicked, D)
        ws = self._ws.get(nb, dev)
        N.call("nrms_user_encode", N.ptr(x), B, n_clicked, x.stride(0), x.stride(1),
               ctypes_byref(w), N.ptr(out), N.ptr(ws), ws.numel(), N.stream_handle(dev))
        return out


class DotProductClickPredictor(nn.Module):
    """src/model/general/click_predictor/dot_product.py:4-19 on the HIP path."""

    def forward(self, candidate_news_vector, user_vector):
        if self.training:  # differentiable (dot_product.py:10-19)
            return torch.bmm(candidate_news_vector, user_vector.unsqueeze(dim=2)).squeeze(dim=2)
        news = _f32(candidate_news_vector)
        user = _f32(user_vector.to(news.device))
        B, C, D = news.shape
        out = torch.empty(B, C, dtype=torch.float32, device=news.device)
        if B * C == 0:
            return out
        N.call("nrms_score", N.ptr(news), B, C, C * D, D, N.ptr(user), D, D, N.ptr(out),
               N.stream_handle(news.device))
        return out


class NRMS(nn.Module):
    """NRMS network (src/model/NRMS/__init__.py:7-84)."""

    def __init__(self, config=NRMSConfig, pretrained_word_embedding=None):
        super().__init__()
        self.config = config
        self.news_encoder = NewsEncoder(config, pretrained_word_embedding)
        self.user_encoder = UserEncoder(config)
        self.click_predictor = DotProductClickPredictor()
        self._ws = _Workspace()
        self._train_calls = 0

    def forward(self, candidate_news, clicked_news):
        """candidate_news: list (1+K) of {"title": LongTensor[B, L]};
        clicked_news: list (N) of the same -> logits [B, 1+K]. One fused
        launch sequence for all B*(1+K+N) titles (src/model/NRMS/__init__.py:19-48).
        In training mode: the autograd path of train.py, dropout included."""
        cand = torch.stack([x["title"] for x in candidate_news], dim=1)
        clk = torch.stack([x["title"] for x in clicked_news], dim=1)
        return self.forward_ids(cand, clk)

    def forward_ids(self, cand_ids, clicked_ids, proj_mode=None):
        """Tensor form of forward: cand_ids [B, C, L], clicked_ids [B, N, L]."""
        ne = self.news_encoder
        if self.training:
            cand, clk = ne._ids(cand_ids), ne._ids(clicked_ids)
            if cand.is_cuda and getattr(self.config, "hip_train", True):
                # HIP train-mode forward + backward kernels (train_hip.py); one
                # dropout seed per call, as torch's RNG advances per call
                from . import train_hip
                self._train_calls += 1
                return train_hip.forward_hip(self, cand, clk, seed=self._train_calls)
            return _train.forward_autograd(self, cand, clk)
        cand = ne._ids(cand_ids)
        clk = ne._ids(clicked_ids)
        B, C, L = cand.shape
        n_clicked = clk.shape[1]
        tab = ne.table()
        V, D = tab.shape
        logits = torch.empty(B, C, dtype=torch.float32, device=tab.device)
        if B == 0 or C == 0:
            return logits
        mode = getattr(self.config, "hip_proj_mode", N.NRMS_PROJ_AUTO) if proj_mode is None else proj_mode
        wn, keep_n = ne.weights()
        wu, keep_u = self.user_encoder.weights()
        nb = N.load().nrms_forward_workspace_size(B, C, n_clicked, L, V, D, mode)
        ws = self._ws.get(nb, tab.device)
        N.call("nrms_forward", N.ptr(cand), N.ptr(clk), B, C, n_clicked, L, N.ptr(tab), V,
               ctypes_byref(wn), ctypes_byref(wu), mode, N.ptr(logits), N.ptr(ws), ws.numel(),
               N.stream_handle(tab.device))
        return logits

    def get_news_vector(self, news):
        return self.news_encoder(news)

    def get_user_vector(self, clicked_news_vector):
        return self.user_encoder(clicked_news_vector)

    def get_prediction(self, news_vector, user_vector):
        return self.click_predictor(news_vector.unsqueeze(dim=0),
                                    user_vector.unsqueeze(dim=0)).squeeze(dim=0)


def ctypes_byref(s):
    import ctypes
    return ctypes.byref(s)
