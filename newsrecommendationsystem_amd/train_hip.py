"""HIP training step of NRMS: the train-mode forward (dropout on) and its
backward as explicit kernels of libnrms_hip.so (include/nrms_hip.h, "Training
kernels"), wrapped in a torch.autograd.Function so that the reference loop
body (src/train.py:202-236: y_pred = model(...); loss = criterion(y_pred, 0);
loss.backward(); optimizer.step()) drives it unchanged.

Forward (news_encoder.py:27-48, user_encoder.py:15-26, dot_product.py:8-19):
  X  = E[ids]                      nrms_embedding_gather
  Xd = dropout(X, p)               nrms_dropout (counter-based mask, seed 2s)
  qkv = Xd [Wq;Wk;Wv]^T + b        nrms_qkv_project (per-token rows)
  ctx = MHSA_rawexp(qkv)           nrms_self_attention
  cd  = dropout(ctx, p)            nrms_dropout (seed 2s+1)
  vec = additive(cd)               nrms_additive_forward_train (keeps tanh y, scores)
  user = additive(MHSA(vec_clicked [Wq;Wk;Wv]_u^T + b_u))
  logits = <vec_cand, user>        nrms_score
Backward: nrms_score_backward -> nrms_additive_backward -> nrms_self_attention_backward
-> nrms_qkv_project_backward (user, then news) -> dropout masks -> nrms_embedding_backward
(dense gradient, row padding_idx = 0 left zero as nn.Embedding(padding_idx=0)).

Dropout masks come from the library's counter-based generator, not torch's
RNG: with p > 0 the trajectory is a different (equally distributed) sample
than the reference's; with p = 0 the step is the reference's arithmetic.
HipAdam is torch.optim.Adam's update on the same state keys (exp_avg,
exp_avg_sq, step), so optimizer state_dicts interchange with the reference's.
"""
import ctypes
import os

import torch

from . import _native as N

D_MODEL, QUERY_DIM = 300, 200


def _zeros_like(t):
    return torch.zeros_like(t, memory_format=torch.contiguous_format)


def encoder_params(enc):
    m, a = enc.multihead_self_attention, enc.additive_attention
    return [m.W_Q.weight, m.W_Q.bias, m.W_K.weight, m.W_K.bias, m.W_V.weight, m.W_V.bias,
            a.linear.weight, a.linear.bias, a.attention_query_vector]


def model_params(model):
    """The 19 parameters in the order NRMSTrain returns gradients for."""
    return ([model.news_encoder.word_embedding.weight] + encoder_params(model.news_encoder)
            + encoder_params(model.user_encoder))


class _Scratch:
    def __init__(self):
        self.bufs = {}

    def get(self, nbytes, dev, slot="main"):
        nbytes = max(int(nbytes), 256)
        buf = self.bufs.get(slot)
        if buf is None or buf.numel() < nbytes or buf.device != dev:
            buf = self.bufs[slot] = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        return buf


_scratch = _Scratch()


class NRMSTrain(torch.autograd.Function):
    @staticmethod
    def forward(ctx, model, cand, clk, p, seed, *params):
        ne, ue = model.news_encoder, model.user_encoder
        E = params[0]
        dev = E.device
        st = N.stream_handle(dev)
        P = N.ptr
        B, C, L = cand.shape
        n_clk = clk.shape[1]
        T = B * (C + n_clk)
        R = T * L
        V, D = E.shape
        Q = ue.additive_attention.linear.out_features
        f32 = dict(dtype=torch.float32, device=dev)
        ids = torch.cat([cand.reshape(B * C, L), clk.reshape(B * n_clk, L)]).contiguous()
        wn, keep_n = ne.weights()
        wu, keep_u = ue.weights()
        ewn, ewu = ctypes.byref(wn), ctypes.byref(wu)
        s1, s2 = 2 * int(seed), 2 * int(seed) + 1

        X = torch.empty(R, D, **f32)
        N.call("nrms_embedding_gather", P(ids), R, P(E.detach()), V, D, P(X), st)
        Xd = torch.empty_like(X)
        N.call("nrms_dropout", P(X), P(Xd), R * D, ctypes.c_float(p), ctypes.c_uint64(s1), st)
        del X
        qkv = torch.empty(R, 3 * D, **f32)
        N.call("nrms_qkv_project", P(Xd), R, None, R, ewn, P(qkv), 0, st)
        cm = torch.empty(R, D, **f32)
        N.call("nrms_self_attention", P(qkv), R, None, T, None, T, L, ewn, P(cm), st)
        cd = torch.empty_like(cm)
        N.call("nrms_dropout", P(cm), P(cd), R * D, ctypes.c_float(p), ctypes.c_uint64(s2), st)
        del cm
        y = torch.empty(R, Q, **f32)
        sc = torch.empty(R, **f32)
        vec = torch.empty(T, D, **f32)                       # [candidates B*C | clicked B*N]
        N.call("nrms_additive_forward_train", P(cd), T, L, ewn, P(y), P(sc), P(vec), st)
        cand_vec, clk_vec = vec[:B * C], vec[B * C:]

        Ru = B * n_clk
        uqkv = torch.empty(Ru, 3 * D, **f32)
        N.call("nrms_qkv_project", P(clk_vec), Ru, None, Ru, ewu, P(uqkv), 0, st)
        uctx = torch.empty(Ru, D, **f32)
        N.call("nrms_self_attention", P(uqkv), Ru, None, B, None, B, n_clk, ewu, P(uctx), st)
        yu = torch.empty(Ru, Q, **f32)
        scu = torch.empty(Ru, **f32)
        user = torch.empty(B, D, **f32)
        N.call("nrms_additive_forward_train", P(uctx), B, n_clk, ewu, P(yu), P(scu), P(user), st)
        logits = torch.empty(B, C, **f32)
        N.call("nrms_score", P(cand_vec), B, C, C * D, D, P(user), D, D, P(logits), st)

        ctx.model = model
        ctx.dims = (B, C, n_clk, L, T, R, V, D, Q)
        ctx.p, ctx.seeds = p, (s1, s2)
        ctx.keep = (wn, keep_n, wu, keep_u)
        ctx.save_for_backward(ids, Xd, qkv, cd, y, sc, vec, uqkv, uctx, yu, scu, user)
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        ids, Xd, qkv, cd, y, sc, vec, uqkv, uctx, yu, scu, user = ctx.saved_tensors
        B, C, n_clk, L, T, R, V, D, Q = ctx.dims
        wn, _, wu, _ = ctx.keep
        ewn, ewu = ctypes.byref(wn), ctypes.byref(wu)
        s1, s2 = ctx.seeds
        p = ctx.p
        dev = Xd.device
        st = N.stream_handle(dev)
        P = N.ptr
        lib = N.load()
        f32 = dict(dtype=torch.float32, device=dev)
        dl = dlogits.contiguous().float()
        Ru = B * n_clk

        # gradient buffers: stacked Q|K|V weight / bias gradients, viewed per parameter
        gWn, gbn = torch.zeros(3 * D, D, **f32), torch.zeros(3 * D, **f32)
        gWu, gbu = torch.zeros(3 * D, D, **f32), torch.zeros(3 * D, **f32)
        gWan, gban, gqn = torch.zeros(Q, D, **f32), torch.zeros(Q, **f32), torch.zeros(Q, **f32)
        gWau, gbau, gqu = torch.zeros(Q, D, **f32), torch.zeros(Q, **f32), torch.zeros(Q, **f32)
        gE = torch.zeros(V, D, **f32)
        ws_b = max(lib.nrms_additive_backward_workspace_size(T, L, D, Q),
                   lib.nrms_additive_backward_workspace_size(B, n_clk, D, Q),
                   lib.nrms_qkv_project_backward_workspace_size(D))
        ws = _scratch.get(ws_b, dev)

        dvec = torch.empty(T, D, **f32)
        duser = torch.empty(B, D, **f32)
        N.call("nrms_score_backward", P(vec[:B * C]), B, C, C * D, D, P(user), D, D, P(dl),
               P(dvec), P(duser), st)
        # user encoder
        ductx = torch.empty(Ru, D, **f32)
        N.call("nrms_additive_backward", P(uctx), B, n_clk, ewu, P(yu), P(scu), P(duser), P(ductx),
               P(gWau), P(gbau), P(gqu), P(ws), ws.numel(), st)
        duqkv = torch.empty(Ru, 3 * D, **f32)
        N.call("nrms_self_attention_backward", P(uqkv), P(ductx), B, n_clk, ewu, P(duqkv), st)
        N.call("nrms_qkv_project_backward", P(vec[B * C:]), Ru, ewu, P(duqkv), P(dvec[B * C:]),
               P(gWu), P(gbu), P(ws), ws.numel(), st)
        # news encoder
        dcd = torch.empty(R, D, **f32)
        N.call("nrms_additive_backward", P(cd), T, L, ewn, P(y), P(sc), P(dvec), P(dcd), P(gWan),
               P(gban), P(gqn), P(ws), ws.numel(), st)
        dcm = torch.empty_like(dcd)
        N.call("nrms_dropout", P(dcd), P(dcm), R * D, ctypes.c_float(p), ctypes.c_uint64(s2), st)
        del dcd
        dqkv = torch.empty(R, 3 * D, **f32)
        N.call("nrms_self_attention_backward", P(qkv), P(dcm), T, L, ewn, P(dqkv), st)
        del dcm
        dXd = torch.empty(R, D, **f32)
        N.call("nrms_qkv_project_backward", P(Xd), R, ewn, P(dqkv), P(dXd), P(gWn), P(gbn), P(ws),
               ws.numel(), st)
        dX = torch.empty_like(dXd)
        N.call("nrms_dropout", P(dXd), P(dX), R * D, ctypes.c_float(p), ctypes.c_uint64(s1), st)
        # deterministic (tokens sorted by id, rows summed in token order)
        ws_e = _scratch.get(lib.nrms_embedding_backward_workspace_size(R, V), dev, slot="embed")
        N.call("nrms_embedding_backward_ws", P(ids), R, P(dX), V, D, 0, P(gE), P(ws_e), ws_e.numel(), st)

        def split(gw, gb):
            return [gw[0:D], gb[0:D], gw[D:2 * D], gb[D:2 * D], gw[2 * D:], gb[2 * D:]]
        grads = ([gE] + split(gWn, gbn) + [gWan, gban, gqn] + split(gWu, gbu) + [gWau, gbau, gqu])
        return (None, None, None, None, None, *grads)


def forward_hip(model, cand_ids, clicked_ids, seed):
    """Train-mode NRMS.forward through the HIP kernels (differentiable)."""
    p = float(model.config.dropout_probability) if model.training else 0.0
    return NRMSTrain.apply(model, cand_ids, clicked_ids, p, int(seed), *model_params(model))


class _AdamTensor(ctypes.Structure):
    """nrms_adam_tensor_t (include/nrms_hip.h)."""
    _fields_ = [("param", ctypes.c_void_p), ("grad", ctypes.c_void_p), ("exp_avg", ctypes.c_void_p),
                ("exp_avg_sq", ctypes.c_void_p), ("numel", ctypes.c_int64),
                ("first_block", ctypes.c_int64)]


class HipAdam(torch.optim.Optimizer):
    """torch.optim.Adam (amsgrad=False, weight_decay=0, maximize=False) on the
    HIP update kernel; same state keys (step, exp_avg, exp_avg_sq), so
    optimizer state_dicts interchange with the reference's
    (src/train.py:127,233). The parameters of a group that share a step count
    (the usual case) are updated by nrms_adam_step_multi: the descriptors go
    to the device by value in the kernel arguments (32 per launch), so nothing
    device-side outlives the launch or depends on the current stream.
    Parameters whose step count differs (a parameter that had no gradient on
    some earlier steps) are updated one nrms_adam_step launch each; so is
    everything when NRMS_ADAM_PER_PARAM is set.

    The update writes parameter memory through raw pointers, which torch does
    not see; step() therefore bumps every updated parameter's version counter,
    as an in-place torch op would, so version-keyed caches (NewsEncoder's
    folded Q|K|V table, nrms.py) see the change."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0,
                 amsgrad=False, *, maximize=False, foreach=None, capturable=False,
                 differentiable=False, fused=None, decoupled_weight_decay=False):
        # torch.optim.Adam's param_group fields, so state_dicts interchange both
        # ways (checkpoint.py); only the reference's configuration is computed
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                                      amsgrad=amsgrad, maximize=maximize, foreach=foreach,
                                      capturable=capturable, differentiable=differentiable,
                                      fused=fused, decoupled_weight_decay=decoupled_weight_decay))
        self._multi = os.environ.get("NRMS_ADAM_PER_PARAM") is None

    @staticmethod
    def _check(p):
        if not (p.is_cuda and p.dtype == torch.float32 and p.is_contiguous()):
            raise TypeError("HipAdam needs contiguous float32 CUDA parameters "
                            f"(got {p.dtype}, device {p.device}, contiguous={p.is_contiguous()})")

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        updated = []
        for group in self.param_groups:
            if group.get("weight_decay", 0) or group.get("amsgrad") or group.get("maximize"):
                raise NotImplementedError("HipAdam computes Adam with weight_decay=0, "
                                          "amsgrad=False, maximize=False (src/train.py:127)")
            b1, b2 = group["betas"]
            args = (ctypes.c_float(group["lr"]), ctypes.c_float(b1), ctypes.c_float(b2),
                    ctypes.c_float(group["eps"]))
            by_step = {}    # (device, step) -> [(p, g, state)]
            for p in group["params"]:
                if p.grad is None:
                    continue
                self._check(p)
                if p.grad.is_sparse:
                    raise RuntimeError("HipAdam does not support sparse gradients")
                state = self.state[p]
                if not state:
                    state["step"] = torch.tensor(0.0)
                    state["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                    state["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                state["step"] += 1
                g = p.grad.float().contiguous()
                by_step.setdefault((p.device, int(state["step"].item())), []).append((p, g, state))
            for (dev, step), live in by_step.items():
                stream = N.stream_handle(dev)
                if self._multi and len(live) > 1:
                    arr = (_AdamTensor * len(live))(*[
                        _AdamTensor(p.data_ptr(), g.data_ptr(), st["exp_avg"].data_ptr(),
                                    st["exp_avg_sq"].data_ptr(), p.numel(), 0)
                        for p, g, st in live])
                    N.call("nrms_adam_step_multi", ctypes.cast(arr, ctypes.c_void_p), len(live),
                           *args, step, stream)
                else:
                    for p, g, st in live:
                        N.call("nrms_adam_step", N.ptr(p), N.ptr(g), N.ptr(st["exp_avg"]),
                               N.ptr(st["exp_avg_sq"]), p.numel(), *args, step, stream)
                updated += [t for p, _, st in live for t in (p, st["exp_avg"], st["exp_avg_sq"])]
        if updated:
            torch.autograd.graph.increment_version(updated)
        return loss
