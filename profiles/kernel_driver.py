"""Run one bench stage in isolation (for rocprofv3 counter passes).

    python profiles/kernel_driver.py <stage> [--iters 10] [--unfused]

Builds the bench workload (B = 1024 impressions, V = 70,976, folded
projection), runs the full forward once, then launches only `<stage>`
`iters` times on the same buffers.
"""
import argparse
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from newsrecommendationsystem_amd import _native as N  # noqa: E402
from newsrecommendationsystem_amd.pipeline import ForwardPlan  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("stage")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--unfused", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    if a.stage == "forward":   # the product path itself (nrms_forward on the bench's stream batch)
        from newsrecommendationsystem_amd import stream as S
        from newsrecommendationsystem_amd.pipeline import TimedForward
        model = bench.build_model(dev)
        idx = bench.stream_impressions(0, 1, 1024, dev)
        cand, clk = S.batch(0, idx, bench.V_WORDS)
        fwd = TimedForward(model, 1024, bench.C, bench.N_CLICKED, bench.L)
        with torch.no_grad():
            for _ in range(a.iters + 1):
                fwd.run(cand, clk)
        torch.cuda.synchronize()
        print("ok", a.stage, a.iters)
        return
    if a.stage == "gather":   # isolated HBM gather figure (bench.gather_hbm)
        for _ in range(a.iters):
            bench.gather_hbm(dev, reps=1)
        torch.cuda.synchronize()
        print("ok", a.stage, a.iters)
        return
    model = bench.build_model(dev)
    cand, clk = bench.synth_impressions(1000, 1024, bench.V_WORDS, dev)
    plan = ForwardPlan(model, 1024, bench.C, bench.N_CLICKED, bench.L, fused=not a.unfused)
    with torch.no_grad():
        plan.run(cand, clk)
        torch.cuda.synchronize()
        B, C, Nc, L, D, V = plan.B, plan.C, plan.N, plan.L, plan.D, plan.V
        n_clk, n_all = B * Nc, B * (C + Nc)
        st = N.stream_handle(dev)
        P = N.ptr
        wn, wu = ctypes.byref(plan.wn), ctypes.byref(plan.wu)
        pws = torch.empty(N.load().nrms_qkv_project_workspace_size(D), dtype=torch.uint8, device=dev)
        calls = {
            # the product path's projection (proj_x6.hip, W split once per call)
            "qkv_news": lambda: N.call("nrms_qkv_project_ws", P(plan.table), V, None, V, wn, P(plan.qkv),
                                       plan.ldq, P(pws), pws.numel(), st),
            "qkv_user": lambda: N.call("nrms_qkv_project_ws", P(plan.news), n_clk, None, n_clk, wu,
                                       P(plan.uqkv), plan.uldq, P(pws), pws.numel(), st),
            # the staged GEMM (gemm_x6_kernel: nrms_qkv_project)
            "qkv_news_staged": lambda: N.call("nrms_qkv_project", P(plan.table), V, None, V, wn, P(plan.qkv),
                                       plan.ldq, st),
            "news_fused": lambda: N.call("nrms_news_attention_pool", P(plan.qkv), plan.ldq, V, P(clk), n_clk,
                                         P(cand), n_all, L, wn, P(plan.news), P(plan.fws),
                                         plan.fws.numel(), st),
            "mhsa_news": lambda: N.call("nrms_self_attention", P(plan.qkv), V, P(clk), n_clk, P(cand), n_all,
                                        L, wn, P(plan.ctx), st),
            "addscore_news": lambda: N.call("nrms_additive_scores", P(plan.ctx), n_all * L, wn, P(plan.scores), st),
            "qkv_user_staged": lambda: N.call("nrms_qkv_project", P(plan.news), n_clk, None, n_clk, wu, P(plan.uqkv),
                                       plan.uldq, st),
            "mhsa_user": lambda: N.call("nrms_self_attention", P(plan.uqkv), n_clk, None, B, None, B, Nc, wu,
                                        P(plan.uctx), st),
        }
        for _ in range(a.iters):
            calls[a.stage]()
        torch.cuda.synchronize()
    print("ok", a.stage, a.iters)


if __name__ == "__main__":
    main()
