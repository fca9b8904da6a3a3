import ctypes, os, sys, numpy as np, torch
sys.path.insert(0, os.getcwd())
from newsrecommendationsystem_amd import _native as N
import bench
dev = torch.device("cuda:0")
model = bench.build_model(dev)
ue = model.user_encoder
w, keep = ue.weights()
out_all = []
for (B, L, scale) in [(1024, 50, 0.3), (37, 50, 0.3), (64, 17, 0.5), (8, 64, 0.3), (16, 5, 0.3), (16, 50, 30.0)]:
    g = torch.Generator(device="cpu").manual_seed(B * 100 + L)
    ld = N.load().nrms_qkv_row_stride(300)
    qkv = (torch.randn(B * L, ld, generator=g) * scale).to(dev)
    out = torch.empty(B, 300, device=dev)
    nb = N.load().nrms_user_attention_pool_workspace_size(B, L, 300)
    ws = torch.zeros(nb, dtype=torch.uint8, device=dev)
    N.call("nrms_user_attention_pool", N.ptr(qkv), ld, B, L, ctypes.byref(w), N.ptr(out), N.ptr(ws), nb, N.stream_handle(dev))
    torch.cuda.synchronize()
    out_all.append(out.cpu().numpy())
np.savez(sys.argv[1], *out_all)
print("ok", [float(np.abs(o).sum()) for o in out_all])
