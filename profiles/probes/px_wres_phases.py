"""Phase cycles of proj_qkv_kernel (s_memtime stamps, probe build):
    bash _ab/build_variant.sh pxt proj_x6.hip -DNRMS_PX_TIMING
    NRMS_LIB_PATH=_ab/lib_pxt.so python profiles/probes/px_phases.py
Runs the bench's vocabulary projection (V = 70,976 rows) through
nrms_qkv_project_ws and prints, per phase, the mean and max over waves of the
cycles summed over the launch (stamps land after the pack in the workspace)."""
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
ne = model.news_encoder
w, keep = ne.weights()
tab = ne.table()
V = tab.shape[0]
ld = N.load().nrms_qkv_row_stride(300)
qkv = torch.empty(V, ld, device=dev)
nb = N.load().nrms_qkv_project_workspace_size(300)
ws = torch.zeros(nb, dtype=torch.uint8, device=dev)
st = N.stream_handle(dev)
for _ in range(3):
    N.call("nrms_qkv_project_ws", N.ptr(tab), V, None, V, ctypes.byref(w), N.ptr(qkv), ld, N.ptr(ws), nb, st)
torch.cuda.synchronize()
stamps = ws[-256 * 8 * 8 * 8:].view(torch.int64).cpu().numpy().reshape(256, 8, 8)   # [WG][wave][phase]
nw = 4
stamps = stamps[:, :nw]
names = ["ng-prologue", "ksteps0-4+split", "ksteps5-9", "epilogue", "barrier", "-", "-", "-"]
tot = stamps.sum(axis=2)
print("%d waves; total cycles per wave: mean %.0f max %.0f" % (nw, tot.mean(), tot.max()))
for k, n in enumerate(names[:5]):
    v = stamps[:, :, k]
    print(f"{n:20s} mean {v.mean():10.0f}  max {v.max():10.0f}")
# per XCD (workgroup b runs on XCD b % 8) and per tile count
tot_wg = tot.max(axis=1)
print("per XCD: mean / max of the workgroup's slowest wave (cycles)")
for x in range(8):
    v = tot_wg[x::8]
    print(f"  XCD {x}: {v.mean():10.0f} {v.max():10.0f}")
n_tiles = (V + 31) // 32
t = np.array([((b + 1) * n_tiles) // 256 - (b * n_tiles) // 256 for b in range(256)])
for k in sorted(set(t.tolist())):
    print(f"  {k} tiles: {tot_wg[t == k].mean():10.0f} ({(t == k).sum()} WGs)")
order = np.argsort(tot_wg)
print("slowest WGs:", order[-10:].tolist(), tot_wg[order[-10:]].astype(int).tolist())
print("per wave (WG 0..3): totals and phases")
for b in range(4):
    print(b, [int(x) for x in tot[b]], [[int(y) for y in stamps[b, w, :5]] for w in range(4)])
print("mean total by wave index:", [int(tot[:, w].mean()) for w in range(4)])
