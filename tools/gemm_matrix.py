"""GEMM-only timing matrix at the benchmark shapes: the fq kernel on int4 weights (with and
without a salient tail), on dense fp16 weights (same kernel, no decode), and the vendor
fp16 GEMM (hipBLASLt via torch).  TFLOP/s on the algorithmic 2*M*N*K.
python tools/gemm_matrix.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd")]
import torch  # noqa: E402

from smoothquant import ops  # noqa: E402

SHAPES = [(16384, 4096, 4096, 128, 0.10), (2048, 4096, 4096, 64, 0.05),
          (2048, 4096, 11008, 64, 0.05), (2048, 11008, 4096, 64, 0.05)]
dev = torch.device("cuda")


def t_ms(fn, it=30, warm_ms=0.0):
    """Average ms per call over `it` calls (HIP events), after 3 calls, or after calling
    for `warm_ms` milliseconds (DVFS: the clock the chip holds under load takes a while)."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    if warm_ms > 0:
        import time
        t0 = time.perf_counter()
        while (time.perf_counter() - t0) * 1e3 < warm_ms:
            for _ in range(10):
                fn()
            torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


def _main():
  for (M, K, N, G, p) in SHAPES:
      g = torch.Generator(device=dev).manual_seed(0)
      w = (torch.randn(N, K, generator=g, device=dev) * 0.02).half()
      x = torch.randn(M, K, generator=g, device=dev).half()
      fl = 2.0 * M * N * K
      row = []
      for label, mode, sal_p in (("int4+tail", "per_group", p), ("int4 S=0", "per_group", 0.0),
                                 ("dense+tail", "none", p), ("dense S=0", "none", 0.0)):
          sal = None
          if sal_p > 0:
              sal = torch.argsort(x.float().abs().mean(0), descending=True)[: int(sal_p * K)].cpu()
          pw = ops.pack_weight(w, mode, 4, G, sal)
          a = ops.quant_act_fp(x, pw, "per_token", 4, G)
          ms = t_ms(lambda: ops.gemm_fq(a, pw, None), it=200, warm_ms=300)
          row.append(f"{label} {fl / ms / 1e9:7.1f}")
      ms = t_ms(lambda: torch.nn.functional.linear(x, w), it=200, warm_ms=300)
      row.append(f"hipBLASLt {fl / ms / 1e9:7.1f}")
      print(f"M={M:5d} K={K:5d} N={N:5d}: " + " | ".join(row) + "  TFLOP/s", flush=True)


if __name__ == "__main__":
    _main()
