"""Diagnostic: A-operand mismatches of ops.quant_act_fp against the oracle over K and data
kinds (tie-heavy small integers vs continuous).  python tools/qa_diag.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import fake_quant_oracle as O  # noqa: E402
from smoothquant import ops  # noqa: E402
from smoothquant.fake_quant import W4A4Linear  # noqa: E402

dev = torch.device("cuda")
TD = {"fp16": torch.float16, "bf16": torch.bfloat16, "fp32": torch.float32}


def bits(a, dtn):
    a = np.asarray(a, np.float32)
    if dtn == "fp32":
        return a.view(np.uint32)
    return a.astype(np.float16).view(np.uint16) if dtn == "fp16" else (a.view(np.uint32) >> 16).astype(np.uint16)


def run(M, K, dtn, p, ties, G=64):
    dt = O.DT(dtn)
    g = np.random.default_rng(K + M)
    raw = g.standard_normal((M, K))
    x = dt.rnd((np.round(raw * 2.0) if ties else raw).astype(np.float32))
    imp = (np.abs(x).mean(0) + g.random(K) * 1e-3).astype(np.float32)
    lin = torch.nn.Linear(K, 128, bias=False).to(dev, TD[dtn])
    q = W4A4Linear.from_float(lin, weight_quant="per_group", act_quant="per_group",
                              importance=torch.from_numpy(imp), salient_prop=p, group_size=G)
    pw = q.packed()
    a = ops.quant_act_fp(torch.from_numpy(x).to(dev, TD[dtn]), pw, "per_group", 4, G)
    a = a.float().cpu().numpy()
    sal = O.select_salient(imp, p)
    qx = O.quantize_input(x, "per_group", 4, G, sal, dt)
    amap = pw.amap.cpu().numpy()
    want = np.zeros_like(a)
    v = amap >= 0
    want[:, :pw.Kp][:, v] = qx[:, amap[v]]
    if sal is not None:
        want[:, pw.Kp:pw.Kp + pw.S] = qx[:, sal]
    bad = np.argwhere(bits(a, dtn) != bits(want, dtn))
    vbad = np.argwhere(a != want)  # values: -0.0 == +0.0
    return len(bad), a.size, f"value mismatches {len(vbad)} {vbad[:3].tolist()}"


KS = [int(k) for k in os.environ.get("QA_KS", "2048,4096,8192,11008,17408").split(",")]
DTS = os.environ.get("QA_DTS", "fp16,fp32").split(",")
for dtn in DTS:
    for K in KS:
        for ties in (True, False):
            for M in (2, 64):
                n, tot, first = run(M, K, dtn, 0.02, ties)
                print(f"lc_off={os.environ.get('SQMP_DISABLE_LC', '0')} {dtn} K={K} M={M} ties={ties}: {n}/{tot} differ {first}", flush=True)
