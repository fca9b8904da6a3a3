"""Phase cycles of fused_user_kernel (s_memtime stamps, probe build):
    bash _ab/build_variant.sh ut user_fused.hip -DNRMS_USER_TIMING
    NRMS_LIB_PATH=_ab/lib_ut.so python profiles/probes/user_phases.py
Runs the UserEncoder tail (nrms_user_attention_pool) of the bench's B = 1024
users (rows from a random q|k|v buffer, every row projected) and prints per
phase the mean / max over workgroups of wave 0's cycles (barrier to barrier)."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from newsrecommendationsystem_amd import _native as N  # noqa: E402
import bench  # noqa: E402

dev = torch.device("cuda:0")
model = bench.build_model(dev)
ue = model.user_encoder
w, keep = ue.weights()
B, L = 1024, 50
ld = N.load().nrms_qkv_row_stride(300)
qkv = (torch.randn(B * L, ld, device=dev) * 0.3)
out = torch.empty(B, 300, device=dev)
nb = N.load().nrms_user_attention_pool_workspace_size(B, L, 300)
ws = torch.zeros(nb, dtype=torch.uint8, device=dev)
st = N.stream_handle(dev)
for _ in range(3):
    N.call("nrms_user_attention_pool", N.ptr(qkv), ld, B, L, ctypes.byref(w), N.ptr(out), N.ptr(ws), nb, st)
torch.cuda.synchronize()
stamps = ws[-4096 * 8 * 8:].view(torch.int64).cpu().numpy().reshape(4096, 8)[:B]
names = ["stage K|V", "attention", "context split", "additive GEMM", "softmax", "pooling"]
print("total cycles per workgroup: mean %.0f max %.0f" % (stamps.sum(1).mean(), stamps.sum(1).max()))
for k, n in enumerate(names):
    print(f"{n:16s} mean {stamps[:, k].mean():9.0f}  max {stamps[:, k].max():9.0f}")
