"""Stage-by-stage NRMS forward over the C ABI, with optional HIP-event timing.

``nrms_forward`` (include/nrms_hip.h) runs the whole scoring path in one call;
ForwardPlan issues the same launches one stage at a time from preallocated
buffers so a harness can bracket each kernel with events on the launch stream
(bench.py uses this for the per-kernel roofline). Output is bitwise identical
to nrms_forward (tests/test_gpu_parity.py::test_plan_matches_forward).

Stage order (forward semantics, src/model/NRMS/__init__.py:19-48):
  qkv_news      Q|K|V projection (folded: whole vocabulary; direct: every token)
  news_fused    raw-exp MHSA + additive attention + pooling of all B*(N+C)
                titles in one kernel (nrms_news_attention_pool); with
                fused=False the three separate stages instead:
                mhsa_news / addscore_news / pool_news
  qkv_user      Q|K|V projection of the clicked news vectors
  user_fused    raw-exp MHSA + additive attention + pooling per user in one
                kernel (nrms_user_attention_pool); with fused=False (or a
                shape the fused kernel does not take): mhsa_user /
                addscore_user / pool_user
  score         dot-product click predictor
"""
import ctypes

import torch

from . import _native as N

D_MODEL = 300


class ForwardPlan:
    def __init__(self, model, B, C, n_clicked, L, proj_mode=N.NRMS_PROJ_FOLDED, fused=True):
        ne = model.news_encoder
        self.model = model
        self.dev = ne.word_embedding.weight.device
        self.table = ne.table()
        self.V, self.D = self.table.shape
        self.B, self.C, self.N, self.L = B, C, n_clicked, L
        n_all = B * (C + n_clicked)
        self.folded = proj_mode == N.NRMS_PROJ_FOLDED or (
            proj_mode == N.NRMS_PROJ_AUTO and n_all * L > self.V)
        f32 = dict(dtype=torch.float32, device=self.dev)
        D = self.D
        qkv_rows = self.V if self.folded else n_all * L
        lib = N.load()
        # rows of nrms_qkv_row_stride for the fused tails, packed 3D rows for the stage kernels
        self.ldq = lib.nrms_qkv_row_stride(D) if fused else 3 * D
        self.uldq = lib.nrms_qkv_row_stride(D) if fused and n_clicked <= 64 else 3 * D
        self.qkv = torch.empty(qkv_rows, self.ldq, **f32)
        self.ctx = torch.empty(n_all * L, D, **f32)
        self.scores = torch.empty(n_all * L, **f32)
        self.news = torch.empty(n_all, D, **f32)        # [clicked B*N | candidates B*C]
        self.uqkv = torch.empty(B * n_clicked, self.uldq, **f32)
        self.uctx = torch.empty(B * n_clicked, D, **f32)
        self.uscores = torch.empty(B * n_clicked, **f32)
        self.user = torch.empty(B, D, **f32)
        self.logits = torch.empty(B, C, **f32)
        # the projections run through nrms_qkv_project_ws (W split once per
        # call), as nrms_forward's: the same rows under every arithmetic
        self.pws = torch.empty(lib.nrms_qkv_project_workspace_size(D), dtype=torch.uint8, device=self.dev)
        self.wn, self._keep_n = ne.weights()
        self.wu, self._keep_u = model.user_encoder.weights()
        self.fused = fused
        self.user_fused = fused and n_clicked <= 64 and D == D_MODEL
        news_st = ["news_fused"] if fused else ["mhsa_news", "addscore_news", "pool_news"]
        user_st = ["user_fused"] if self.user_fused else ["mhsa_user", "addscore_user", "pool_user"]
        self.stages = ["qkv_news"] + news_st + ["qkv_user"] + user_st + ["score"]
        if fused:
            nb = lib.nrms_news_attention_pool_workspace_size(n_all, L, D)
            self.fws = torch.empty(nb, dtype=torch.uint8, device=self.dev)
        if self.user_fused:
            nb = lib.nrms_user_attention_pool_workspace_size(B, n_clicked, D)
            self.uws = torch.empty(nb, dtype=torch.uint8, device=self.dev)
            # the clicked positions' all-padding flags, computed into these
            # buffers before the first stage event (no allocation per call)
            self._eq = torch.empty(B, n_clicked, L, dtype=torch.bool, device=self.dev)
            self._pad = torch.empty(B, n_clicked, dtype=torch.bool, device=self.dev)

    def run(self, cand_ids, clicked_ids, events=None):
        """cand_ids [B,C,L], clicked_ids [B,N,L] int64 on the device. If
        ``events`` (len(stages)+1 torch.cuda.Event) is given, event i is
        recorded before stage i and the last one after the final stage."""
        B, C, Nc, L, D, V = self.B, self.C, self.N, self.L, self.D, self.V
        n_clk, n_all = B * Nc, B * (C + Nc)
        st = N.stream_handle(self.dev)
        wn, wu = ctypes.byref(self.wn), ctypes.byref(self.wu)
        P = N.ptr
        rec = (lambda i: events[i].record()) if events is not None else (lambda i: None)
        if self.user_fused:
            # the clicked positions holding all-padding titles (one news vector):
            # the user tail compacts them as nrms_forward does (token compaction)
            torch.eq(clicked_ids, 0, out=self._eq)
            torch.all(self._eq, dim=-1, out=self._pad)

        rec(0)
        ldq, uldq = self.ldq, self.uldq
        pws, npws = P(self.pws), self.pws.numel()
        if self.folded:
            N.call("nrms_qkv_project_ws", P(self.table), V, None, V, wn, P(self.qkv), ldq, pws, npws, st)
        else:
            N.call("nrms_qkv_project_ws", P(self.table), V, P(clicked_ids), n_clk * L, wn,
                   P(self.qkv), ldq, pws, npws, st)
            tail = self.qkv[n_clk * L:]
            N.call("nrms_qkv_project_ws", P(self.table), V, P(cand_ids), B * C * L, wn, P(tail), ldq,
                   pws, npws, st)
        rec(1)
        k = 1
        rows, ia, ib = (V, P(clicked_ids), P(cand_ids)) if self.folded else (n_all * L, None, None)
        if self.fused:
            N.call("nrms_news_attention_pool", P(self.qkv), ldq, rows, ia, n_clk, ib, n_all, L, wn,
                   P(self.news), P(self.fws), self.fws.numel(), st)
        else:
            N.call("nrms_self_attention", P(self.qkv), rows, ia, n_clk, ib, n_all, L, wn,
                   P(self.ctx), st)
            rec(k + 1)
            N.call("nrms_additive_scores", P(self.ctx), n_all * L, wn, P(self.scores), st)
            rec(k + 2)
            N.call("nrms_additive_pool", P(self.ctx), P(self.scores), n_all, L, D, P(self.news), st)
            k += 2
        k += 1
        rec(k)
        N.call("nrms_qkv_project_ws", P(self.news), n_clk, None, n_clk, wu, P(self.uqkv), uldq, pws, npws, st)
        rec(k + 1)
        if self.user_fused:
            N.call("nrms_user_attention_pool_padded", P(self.uqkv), uldq, B, Nc, P(self._pad), wu, P(self.user),
                   P(self.uws), self.uws.numel(), st)
            k += 1
        else:
            N.call("nrms_self_attention", P(self.uqkv), n_clk, None, B, None, B, Nc, wu,
                   P(self.uctx), st)
            rec(k + 2)
            N.call("nrms_additive_scores", P(self.uctx), n_clk, wu, P(self.uscores), st)
            rec(k + 3)
            N.call("nrms_additive_pool", P(self.uctx), P(self.uscores), B, Nc, D, P(self.user), st)
            k += 3
        rec(k + 1)
        N.call("nrms_score", P(self.news[n_clk:]), B, C, C * D, D, P(self.user), D, D,
               P(self.logits), st)
        rec(k + 2)
        return self.logits

    # Algorithmic work per launch of each stage (SURVEY §8d conventions:
    # GEMMs 2·M·N·K; bytes = operands the stage must read + results it writes).
    def work(self, titles_encoded=None, user_rows_projected=None, news_rows=None, user_rows=None):
        """titles_encoded: titles the fused news tail actually encodes (with
        padding-title dedupe: the titles with a real token + one all-padding
        title); user_rows_projected: clicked rows the UserEncoder's Q|K|V GEMM
        projects (with dedupe: all but the copied padding rows); news_rows:
        (sum of Le, sum of Le^2) over the encoded titles, Le = the distinct q|k|v
        rows a title is encoded on (token compaction: real tokens + one padding
        row; L without it); user_rows: (sum of Le, sum of Le^2) over the users
        (UserEncoder compaction: real history positions + one padding row);
        default all titles, L rows each, and N rows per user."""
        B, C, Nc, L, D, V = self.B, self.C, self.N, self.L, self.D, self.V
        Q, H, dk = 200, 15, D // 15
        n_all, n_clk = B * (C + Nc), B * Nc
        n_enc = n_all if titles_encoded is None else titles_encoded
        n_up = n_clk if user_rows_projected is None else user_rows_projected
        rows, rows_sq = (n_enc * L, n_enc * L * L) if news_rows is None else news_rows
        urows, urows_sq = (n_clk, B * Nc * Nc) if user_rows is None else user_rows
        att_flop = lambda seqs, l: seqs * H * 2 * (2 * l * l * dk)
        qkv_m = V if self.folded else n_all * L
        return {
            "qkv_news": dict(flop=2 * qkv_m * D * 3 * D, split=dict(gemm=2 * qkv_m * D * 3 * D),
                             bytes=4 * (qkv_m * D + qkv_m * 3 * D + 3 * D * D)),
            # gathered q|k|v rows + ids + context rows written
            "mhsa_news": dict(flop=att_flop(n_all, L),
                              bytes=n_all * L * (4 * 3 * D + (8 if self.folded else 0) + 4 * D)),
            "addscore_news": dict(flop=2 * n_all * L * D * Q, bytes=4 * (n_all * L * (D + 1) + Q * D)),
            "pool_news": dict(flop=2 * n_all * L * D, bytes=4 * (n_all * L * (D + 1) + n_all * D)),
            # fused tail: gathered q|k|v rows + ids in, news vectors out, W_add
            # (the context tile stays in LDS)
            # (per title on Le rows: attention 2 contractions x H heads x 2 Le^2 dk,
            # additive GEMM 2 Le D Q, pooling 2 Le D)
            "news_fused": dict(flop=H * 4 * rows_sq * dk + 2 * rows * D * Q + 2 * rows * D,
                               bytes=rows * 4 * 3 * D + n_enc * L * (8 if self.folded else 0)
                               + 4 * (n_all * D + Q * D),
                               split=dict(attention=H * 4 * rows_sq * dk, gemm=2 * rows * D * Q,
                                          pool=2 * rows * D)),
            "qkv_user": dict(flop=2 * n_up * D * 3 * D, bytes=4 * (n_up * 4 * D + 3 * D * D),
                             split=dict(gemm=2 * n_up * D * 3 * D)),
            "mhsa_user": dict(flop=att_flop(B, Nc), bytes=4 * n_clk * 4 * D),
            "addscore_user": dict(flop=2 * n_clk * D * Q, bytes=4 * (n_clk * (D + 1) + Q * D)),
            "pool_user": dict(flop=2 * n_clk * D, bytes=4 * (n_clk * (D + 1) + B * D)),
            # fused user tail: q|k|v rows in, user vectors out (context stays in LDS)
            "user_fused": dict(flop=H * 4 * urows_sq * dk + 2 * urows * D * Q + 2 * urows * D,
                               bytes=4 * (urows * 3 * D + B * D + Q * D),
                               split=dict(attention=H * 4 * urows_sq * dk, gemm=2 * urows * D * Q,
                                          pool=2 * urows * D)),
            "score": dict(flop=2 * B * C * D, bytes=4 * (B * C * D + B * D + B * C)),
        }


class TimedForward:
    """The product path, nrms_forward, with per-stage HIP events
    (nrms_forward_timed): one C-ABI call per step from a preallocated
    workspace; event i is recorded on the launch stream before stage i
    (stages = nrms_forward_stage_name) and the last after the final stage.
    Unlike ForwardPlan it takes nrms_forward's internal shortcuts (the
    UserEncoder's row-list projection after padding-title dedupe)."""

    def __init__(self, model, B, C, n_clicked, L, proj_mode=N.NRMS_PROJ_FOLDED):
        ne = model.news_encoder
        self.dev = ne.word_embedding.weight.device
        self.table = ne.table()
        self.V, self.D = self.table.shape
        self.B, self.C, self.N, self.L, self.mode = B, C, n_clicked, L, proj_mode
        lib = N.load()
        nb = lib.nrms_forward_workspace_size(B, C, n_clicked, L, self.V, self.D, proj_mode)
        self.ws = torch.empty(nb, dtype=torch.uint8, device=self.dev)
        self.logits = torch.empty(B, C, dtype=torch.float32, device=self.dev)
        self.wn, self._keep_n = ne.weights()
        self.wu, self._keep_u = model.user_encoder.weights()
        self.stages = [lib.nrms_forward_stage_name(i).decode() for i in range(N.NRMS_FORWARD_STAGES)]

    def make_events(self, n_steps):
        """n_steps lists of len(stages)+1 timing events, created (recorded once)."""
        evs = [[torch.cuda.Event(enable_timing=True) for _ in range(len(self.stages) + 1)]
               for _ in range(n_steps)]
        for row in evs:
            for e in row:
                e.record()
        torch.cuda.synchronize(self.dev)
        return evs

    def run(self, cand_ids, clicked_ids, events=None):
        arr = None
        if events is not None:
            arr = (ctypes.c_void_p * len(events))(*[ctypes.c_void_p(e.cuda_event) for e in events])
        N.call("nrms_forward_timed", N.ptr(cand_ids), N.ptr(clicked_ids), self.B, self.C, self.N,
               self.L, N.ptr(self.table), self.V, ctypes.byref(self.wn), ctypes.byref(self.wu),
               self.mode, N.ptr(self.logits), N.ptr(self.ws), self.ws.numel(),
               N.stream_handle(self.dev), arr, len(events) if events is not None else 0)
        return self.logits
