"""CPU: sqmp_gemm_h2d's eligibility guards (no GPU needed).  The kernel addresses both
activation planes of a tile through 32-bit buffer offsets, so the host only takes the h2d path
while 2 planes x roundup(M, 128) rows x L halves stay under 4 GiB; larger batches run the
fp32 operand + sqmp_gemm_h2."""
import torch

from smoothquant import ops


def test_h2d_row_guard():
    assert ops._h2d_rows_ok(16384, 4160)          # config 2 in fp32
    assert ops._h2d_rows_ok(2048, 8640)           # OPT-1.3B fc2 at 2048 tokens
    assert not ops._h2d_rows_ok(262144, 4160)     # 4.4 GB of planes
    assert ops._h2d_rows_ok(0, 64)
    # the weight planes too: 2 planes x roundup(N, 256) rows x L halves under 4 GiB
    assert ops._h2d_rows_ok(2048, 4160, 4096)
    assert not ops._h2d_rows_ok(2048, 16384, 65536)


def test_h2_planes_ok_requires_fp32_and_shape():
    class PW:  # the fields h2_planes_ok reads
        dtype = torch.float32
        Kp, S_pad, N, K, S = 4096, 448, 4096, 4096, 409
    assert ops.h2_planes_ok(PW, "per_group", 16384) == (ops.H2D and ops.F32_GEMM == "h2")
    assert not ops.h2_planes_ok(PW, "per_tensor", 16384)
    assert not ops.h2_planes_ok(PW, "per_group", 1 << 20)
    # an empty batch takes the fp32-operand path (the planes would be a 0-row allocation)
    assert not ops.h2_planes_ok(PW, "per_group", 0)
    # the wave quantizer's row buffer: 4 K + 12 per group bytes within 160 KiB
    assert ops.h2_planes_ok(PW, "per_group", 16384, 128) == (ops.H2D and ops.F32_GEMM == "h2")
    PW.K, PW.Kp = 40960, 40960
    assert not ops.h2_planes_ok(PW, "per_group", 16384, 128)
    PW.K, PW.Kp = 4096, 4096
    PW.dtype = torch.float16
    assert not ops.h2_planes_ok(PW, "per_group", 16384)
