"""Debug sweep: A operand of ops.quant_act_fp vs the CPU oracle over (M, K, G, mode)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd")]
import numpy as np, torch
from smoothquant import ops
from smoothquant.fake_quant import W4A4Linear
from oracle import fake_quant_oracle as O
dev = torch.device("cuda")
dt = O.DT("fp16")
for act in ("per_group", "per_token"):
    for M in (128, 256, 512, 1024, 2048):
        for K in (4096,):
            for G in (64,):
                g = torch.Generator(device=dev).manual_seed(K + M)
                lin = torch.nn.Linear(K, 256, bias=False).to(dev, torch.float16)
                x = torch.randn(M, K, generator=g, device=dev).half()
                q = W4A4Linear.from_float(lin, weight_quant="per_group", act_quant=act,
                                          importance=x.float().abs().mean(0).cpu(),
                                          salient_prop=0.05, group_size=G)
                pw = q.packed()
                a = ops.quant_act_fp(x, pw, act, 4, G).float().cpu().numpy()
                amap, sal = pw.amap.cpu().numpy(), pw.salient.cpu().numpy().astype(np.int64)
                qx = O.quantize_input(x.float().cpu().numpy().astype(np.float16), act, 4, G, sal, dt).astype(np.float32)
                want = np.zeros_like(a)
                v = amap >= 0
                want[:, :pw.Kp][:, v] = qx[:, amap[v]]
                want[:, pw.Kp:pw.Kp + pw.S] = qx[:, sal]
                bad = int((a != want).sum())
                print(f"{act:20s} M={M:3d} K={K:5d} G={G:4d}: mismatches {bad}")
