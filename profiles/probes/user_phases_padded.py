"""Phase cycles of fused_user_kernel on the bench's history distribution
(token compaction on: histories of U{1..50} real titles, left-padded with one
shared padding vector, so a user runs on L = real + 1 rows):
    bash _ab/build_variant.sh ut user_fused.hip -DNRMS_USER_TIMING
    NRMS_LIB_PATH=_ab/lib_ut.so python profiles/probes/user_phases_padded.py
Prints per phase the mean over workgroups of wave 0's cycles, overall and by
L range (nrms_user_attention_pool_padded, B = 1024, N = 50)."""
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
w, keep = model.user_encoder.weights()
B, L = 1024, 50
lib = N.load()
ld = lib.nrms_qkv_row_stride(300)
rng = np.random.default_rng(11)
real = rng.integers(1, L + 1, B)
flags = np.zeros((B, L), np.uint8)
for b in range(B):
    flags[b, : L - real[b]] = 1
qkv = torch.randn(B * L, ld, device=dev) * 0.3
padrow = torch.randn(ld, device=dev) * 0.3
fl = torch.from_numpy(flags.reshape(-1)).to(dev)
qkv[fl.bool()] = padrow
out = torch.empty(B, 300, device=dev)
nb = lib.nrms_user_attention_pool_workspace_size(B, L, 300)
ws = torch.zeros(nb, dtype=torch.uint8, device=dev)
st = N.stream_handle(dev)
prev = lib.nrms_set_token_compaction(1)
for _ in range(3):
    N.call("nrms_user_attention_pool_padded", N.ptr(qkv), ld, B, L, N.ptr(fl), ctypes.byref(w), N.ptr(out),
           N.ptr(ws), nb, st)
torch.cuda.synchronize()
lib.nrms_set_token_compaction(prev)
stamps = ws[-4096 * 8 * 8:].view(torch.int64).cpu().numpy().reshape(4096, 8)[:B]
names = ["stage K|V", "attention", "context split", "additive GEMM", "softmax", "pooling"]
rows = np.where(real < L, real + 1, L)
print("total cycles per workgroup: mean %.0f max %.0f (rows per user: mean %.1f)" %
      (stamps.sum(1).mean(), stamps.sum(1).max(), rows.mean()))
for k, n in enumerate(names):
    print(f"{n:16s} mean {stamps[:, k].mean():9.0f}  max {stamps[:, k].max():9.0f}")
for lo, hi in ((1, 16), (17, 32), (33, 51)):
    m = (rows >= lo) & (rows <= hi)
    print(f"L {lo:2d}..{hi:2d} ({m.sum():4d} users): " + "  ".join(
        f"{n.split()[0]} {stamps[m, k].mean():7.0f}" for k, n in enumerate(names)) +
        f"  total {stamps[m].sum(1).mean():7.0f}")
