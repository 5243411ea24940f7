"""Stage-0 register operands of the persistent fqt7 kernel (diag build SQMP_PERSIST_DBG & 256)
against the operand tensors, next to which 32-token slices of y came out wrong."""
import ctypes
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "smoothquant-mixedprecision_amd"))
from test_gpu_fqt import _layer  # noqa: E402
from smoothquant import ops  # noqa: E402
import smoothquant._lib as L  # noqa: E402

M, K, N = 16384, 4096, 4096
dev = torch.device("cuda:0")
q, lin, x = _layer(dev, M, K, N, 128, 0.10, torch.float16)
pw = q.packed()
c4 = ops.quant_act_c4(x, pw, "per_group", 4, 128)
ys = {}
for v in ("3", "67"):
    os.environ["SQMP_FQT7_OPT"] = v
    L.reload_knobs()
    ys[v] = ops.gemm_fqt(*c4, pw, lin.bias, 128).clone()
    torch.cuda.synchronize()
ne = (ys["3"] != ys["67"])
print("differ", int(ne.sum()))
lib = ctypes.CDLL(os.environ["SQMP_LIB_PATH"])
buf = np.zeros(256 * 8 * 64 * 12, np.uint32)
assert lib.sqmp_diag_p67(buf.ctypes.data_as(ctypes.c_void_p)) == 0
d = buf.reshape(256, 8, 64, 12)
codes = c4[0].contiguous().view(torch.int32).reshape(-1).cpu().numpy().view(np.uint32)
sc = c4[1].contiguous().view(torch.int16).cpu().numpy().view(np.uint16)  # [nblk, ngw, 32]
nkm = c4[0].shape[1] * 2 // 64
print("nkm", nkm, "scales", sc.shape)
nbad_c = nbad_s = 0
for wg in range(256):
    for w in range(8):
        nb = int(d[wg, w, 0, 5])
        m0 = int(d[wg, w, 0, 7])
        tn = nb // 8
        exp_c = np.stack([codes[nb * nkm * 256 + l * 4: nb * nkm * 256 + l * 4 + 4] for l in range(64)])
        got_c = d[wg, w, :, 0:4]
        r16 = np.arange(64) & 15
        exp_s = sc[nb, 0, 2 * r16].astype(np.uint32) | (sc[nb, 0, 2 * r16 + 1].astype(np.uint32) << 16)
        got_s = d[wg, w, :, 4]
        okc = (exp_c == got_c).all()
        oks = (exp_s == got_s).all()
        ybad = bool(ne[tn * 256 + w * 32: tn * 256 + w * 32 + 32, m0: m0 + 256].any())
        if not okc or not oks or ybad:
            nbad_c += not okc
            nbad_s += not oks
            if wg < 40:
                print(f"wg {wg} wave {w} tile {int(d[wg, w, 0, 6])} nb {nb} m0 {m0}: codes ok {okc} scales ok {oks} y bad {ybad}",
                      "A0", [hex(v) for v in d[wg, w, 0, 8:12]], "s", hex(int(got_s[0])), hex(int(exp_s[0])))
print("codes wrong", nbad_c, "scales wrong", nbad_s)
