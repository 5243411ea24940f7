"""Where the persistent activation-order grid (SQMP_FQT7_OPT=67) differs from the default
launch: per 256 x 256 output tile, the count of differing elements and the max |diff|."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "smoothquant-mixedprecision_amd"))
from test_gpu_fqt import _layer  # noqa: E402

M, K, N = (int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (16384, 4096, 4096)))
dev = torch.device("cuda:0")
from smoothquant import ops  # noqa: E402
import smoothquant._lib as L  # noqa: E402
q, lin, x = _layer(dev, M, K, N, 128, 0.10, torch.float16)
pw = q.packed()
c4 = ops.quant_act_c4(x, pw, "per_group", 4, 128)
print("operand dims", c4[1].dim(), [tuple(t.shape) for t in c4[:3]])
outs = {}
for v in ("3", "67", "3", "67"):
    os.environ["SQMP_FQT7_OPT"] = v
    L.reload_knobs()
    y = ops.gemm_fqt(*c4, pw, lin.bias, 128).clone()
    torch.cuda.synchronize()
    outs.setdefault(v, []).append(y)
for v, ys in outs.items():
    print(v, "repeatable", torch.equal(ys[0], ys[1]))
a, b = outs["3"][0].float(), outs["67"][0].float()
d = (a - b).abs()
ne = a != b
print("differ", int(ne.sum()), "of", ne.numel(), "max", float(d.max()), "ref max", float(a.abs().max()))
T = 256
tm, tn = (M + T - 1) // T, (N + T - 1) // T
for i in range(tm):
    row = []
    for j in range(tn):
        blk = ne[i * T:(i + 1) * T, j * T:(j + 1) * T]
        row.append(int(blk.sum()))
    if any(row):
        print("tok tile", i, row)
# within a differing tile: which rows/cols
idx = ne.nonzero()
if len(idx):
    print("first diffs", idx[:16].tolist())
    print("token rows differing (mod 256) histogram", torch.bincount(idx[:, 0] % 256, minlength=256)[:64].tolist())
    print("col (weight row) mod 256 hist", torch.bincount(idx[:, 1] % 256, minlength=256)[:64].tolist())
# the first bad tiles in detail: bad 32-token blocks (a wave's register operand) and bad
# 32-weight-row blocks
shown = 0
for i in range(tm):
    for j in range(tn):
        blk = ne[i * T:(i + 1) * T, j * T:(j + 1) * T]
        if blk.any() and shown < 4:
            shown += 1
            tokb = blk.reshape(8, 32, T).any(2).any(1).int().tolist()
            wb = blk.reshape(T, 8, 32).any(2).any(0).int().tolist()
            print(f"tile tok {i} w {j}: bad tok blocks {tokb} bad w blocks {wb} n={int(blk.sum())}")
# one bad 32-token block in detail
done = False
for i in range(tm):
    for j in range(tn):
        blk = ne[i * T:(i + 1) * T, j * T:(j + 1) * T]
        if done or not blk.any():
            continue
        tb = int(blk.reshape(8, 32, T).any(2).any(1).int().argmax())
        r0, c0 = i * T + tb * 32, j * T
        A = a[r0:r0 + 32, c0:c0 + T]
        B = b[r0:r0 + 32, c0:c0 + T]
        D = B - A
        print("block rows", r0, "cols", c0)
        print(" diff mean over tokens per col (first 8):", D.mean(0)[:8].tolist())
        print(" diff std over tokens per col (first 8):", D.std(0)[:8].tolist())
        print(" ratio B/A median", float((B / A.where(A.abs() > 0.5, torch.ones_like(A))).median()))
        # does B equal A of another token block / another column block?
        for dr in range(-256, 257, 32):
            rr = r0 + dr
            if 0 <= rr and rr + 32 <= a.shape[0] and dr != 0:
                if torch.equal(B, a[rr:rr + 32, c0:c0 + T]):
                    print(" equals ref rows", rr)
        print(" A[0,:6]", A[0, :6].tolist())
        print(" B[0,:6]", B[0, :6].tolist())
        done = True
# which K stages explain the bad block: D = sum_k c_k C_k (C_k the 64-position stage product)
from test_gpu_fqt import decode_c4, untile_c4  # noqa: E402
codes, scales, xs, wp = c4
Kq = (pw.K - pw.S + 63) // 64 * 64
cr, sr, xr = untile_c4(codes, scales, xs, M, Kq, pw.S_pad)
X = torch.cat([decode_c4(cr, sr, Kq, 128, torch.float16).float(), xr.float()], 1)
Wf = wp[:N].float()
print("X", tuple(X.shape), "W", tuple(Wf.shape))
yr = X.double() @ Wf.double().t() + lin.bias.double()
print("ref check rel", float((yr - a.double()).norm() / yr.norm()))
nst = X.shape[1] // 64
shown = 0
for i in range(tm):
    for j in range(tn):
        blk = ne[i * T:(i + 1) * T, j * T:(j + 1) * T]
        if shown >= 3 or not blk.any():
            continue
        for tb in range(8):
            if not blk[tb * 32:(tb + 1) * 32].any() or shown >= 3:
                continue
            shown += 1
            r0, c0 = i * T + tb * 32, j * T
            D = (b - a)[r0:r0 + 32, c0:c0 + T].double().reshape(-1)
            Cs = torch.stack([(X[r0:r0 + 32, 64 * k:64 * k + 64].double() @
                               Wf[c0:c0 + T, 64 * k:64 * k + 64].double().t()).reshape(-1)
                              for k in range(nst)], 1)
            c = torch.linalg.lstsq(Cs, D.unsqueeze(1)).solution.squeeze(1)
            res = float((Cs @ c - D).norm() / D.norm())
            top = c.abs().argsort(descending=True)[:6].tolist()
            print(f"block r{r0} c{c0}: nst {nst} (codes {Kq // 64}) resid {res:.3f} top",
                  [(k, round(float(c[k]), 3)) for k in top])
