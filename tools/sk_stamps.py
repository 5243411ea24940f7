"""Where the stream-K grouped GEMM's time goes: per-workgroup, per-segment real-time stamps
(100 MHz) of the diagnostics build (SQMP_DIAG=1 build_ext.py; gemm_fq7_kernel's SK_STAMP
points: segment start, K loop done, hand-off done, segment end), for the Llama-2-7B q/k/v and
gate/up grouped launches at 2048 tokens.

    SQMP_LIB_PATH=ab_tmp/diag.so python tools/sk_stamps.py

Per shape: the kernel's span (first start -> last end) and the spread of workgroup end times;
per segment role (0 whole tile, 1 second part, 2 first part) the median / 90th percentile of
its K loop, hand-off and epilogue times (us)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from smoothquant import ops  # noqa: E402
from smoothquant._lib import load  # noqa: E402
from test_gpu_sibling import _siblings  # noqa: E402

lib = load()
f = lib.sqmp_diag_sk_stamps
f.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
f.restype = ctypes.c_int
dev = torch.device("cuda")

for name, M, K, Ns in (("qkv", 2048, 4096, (4096, 4096, 4096)), ("gate_up", 2048, 4096, (11008, 11008))):
    layers, x = _siblings(dev, M, K, Ns, 64, 0.05, torch.float16, seed=21)
    pws = [q.packed() for q in layers]
    a = ops.quant_act_fp_group(x, pws, "per_group", 4, 64)
    biases = [q.bias.reshape(-1) for q in layers]
    for _ in range(20):
        ops.gemm_fq7_group(a, pws, biases)
    torch.cuda.synchronize()
    assert f(None, None) == 0
    torch.cuda.synchronize()
    ops.gemm_fq7_group(a, pws, biases)
    torch.cuda.synchronize()
    st = np.zeros((512, 16), dtype=np.uint64)
    ro = np.zeros((512, 4), dtype=np.int32)
    assert f(st.ctypes.data, ro.ctypes.data) == 0
    st = st.astype(np.int64)
    used = st[:, 0] > 0
    t0 = st[used][:, 0].min()
    ends = []
    per = {0: [], 1: [], 2: []}
    for w in np.nonzero(used)[0]:
        last = 0
        for s in range(4):
            if st[w, 4 * s] == 0 or ro[w, s] < 0:
                break
            a0, a1, a2, a3 = (st[w, 4 * s + k] for k in range(4))
            per[int(ro[w, s])].append(((a1 - a0) / 100, (a2 - a1) / 100, (a3 - a2) / 100, (a0 - t0) / 100))
            last = a3
        ends.append((last - t0) / 100)
    ends = np.array(ends)
    print(f"{name}: {used.sum()} workgroups, span {ends.max():.1f} us, end times median "
          f"{np.median(ends):.1f} p10 {np.percentile(ends, 10):.1f} p90 {np.percentile(ends, 90):.1f} us")
    for r, rows in per.items():
        if not rows:
            continue
        v = np.array(rows)
        print(f"   role {r}: {len(rows):4d} segments  K loop median {np.median(v[:, 0]):6.1f} p90 "
              f"{np.percentile(v[:, 0], 90):6.1f}  hand-off median {np.median(v[:, 1]):5.2f} p90 "
              f"{np.percentile(v[:, 1], 90):5.2f}  epilogue median {np.median(v[:, 2]):5.2f} p90 "
              f"{np.percentile(v[:, 2], 90):5.2f}  start median {np.median(v[:, 3]):6.1f}")
    # a few workgroups' timelines
    for w in list(np.nonzero(used)[0][:3]):
        segs = []
        for s in range(4):
            if st[w, 4 * s] == 0 or ro[w, s] < 0:
                break
            segs.append(f"r{ro[w, s]}[{(st[w, 4 * s] - t0) / 100:.1f}->{(st[w, 4 * s + 1] - t0) / 100:.1f}"
                        f"->{(st[w, 4 * s + 2] - t0) / 100:.1f}->{(st[w, 4 * s + 3] - t0) / 100:.1f}]")
        print(f"   wg {w}: " + " ".join(segs))
