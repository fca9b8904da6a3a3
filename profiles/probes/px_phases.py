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
nw = 8 if stamps[:, 4:].any() else 4
stamps = stamps[:, :nw]
names = ["loop/restage-tail", "setup+kstep0", "ksteps1-9", "epilogue", "barrier1", "A-wait+split", "barrier2", "-"]
tot = stamps.sum(axis=2)
print("%d waves; total cycles per wave: mean %.0f max %.0f" % (nw, tot.mean(), tot.max()))
for k, n in enumerate(names[:7]):
    v = stamps[:, :, k]
    print(f"{n:20s} mean {v.mean():10.0f}  max {v.max():10.0f}")
# per-workgroup busy cycles (max over its waves): the static item ranges' balance
wg = tot.max(axis=1)
print("workgroup totals: min %.0f p10 %.0f median %.0f p90 %.0f max %.0f mean %.0f (max/mean %.4f)"
      % (wg.min(), np.percentile(wg, 10), np.median(wg), np.percentile(wg, 90), wg.max(), wg.mean(), wg.max() / wg.mean()))
# by XCD (workgroups b, b + 8, .. share one: MI355X_MICROARCH.md dispatch notes)
# and by position in the grid
for x in range(8):
    v = wg[x::8]
    print("xcd-slot %d: mean %.0f max %.0f" % (x, v.mean(), v.max()))
q = len(wg) // 4
print("grid quarters (mean):", " ".join("%.0f" % wg[i * q:(i + 1) * q].mean() for i in range(4)))
# per wave class: waves 0-3 hold three N tiles per item, waves 4-7 two
if nw == 8:
    for lo, hi, tag in ((0, 4, "waves 0-3 (3 tiles)"), (4, 8, "waves 4-7 (2 tiles)")):
        v = stamps[:, lo:hi]
        print(tag + ": " + " ".join("%s=%.0f" % (names[k], v[:, :, k].mean()) for k in range(7)))
