"""CPU-only checks of the drop-in boundary: the C-ABI library builds/loads, exports every
symbol include/sqmp_w4a4.h declares, its host-only entry points behave, and the Python
surface mirrors the reference's API and error conventions.  No kernel is launched."""
import ctypes
import inspect
import os
import re

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "sqmp_w4a4.h")


def _declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(sqmp_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    from smoothquant import _lib
    if not os.path.exists(_lib.LIB_PATH):
        import build_ext
        build_ext.build()
    return _lib.load()


def test_header_symbols_exported(lib):
    from smoothquant import _lib
    declared = _declared_functions()
    assert len(declared) >= 12
    for name in declared:
        assert hasattr(lib, name), f"{name} declared in sqmp_w4a4.h but not exported"
        assert name in _lib.SIGNATURES, f"{name} has no ctypes signature"
    assert set(_lib.SIGNATURES) == set(declared)


def test_version_and_status(lib):
    assert b"gfx950" in lib.sqmp_version()
    assert lib.sqmp_status_string(0) == b"ok"
    assert lib.sqmp_status_string(-1) == b"invalid argument"


def _geom(lib, K, S, wmode, G):
    out = [ctypes.c_int() for _ in range(4)]
    st = lib.sqmp_weight_geometry(K, S, wmode, G, *[ctypes.byref(o) for o in out])
    return st, tuple(o.value for o in out)


def test_weight_geometry(lib):
    # per_group (sorted): groups over all K columns, padded to the 128-code K tile; the
    # salient tail padded to 64
    assert _geom(lib, 4096, 409, 2, 128) == (0, (4096, 128, 32, 448))
    assert _geom(lib, 11008, 550, 2, 64) == (0, (11008, 64, 172, 576))
    # G=1024 on K=11008: 11 groups, 256 zero-padding columns in the last (fake_quant.py:176-180)
    assert _geom(lib, 11008, 0, 2, 1024) == (0, (11264, 1024, 11, 0))
    # per_channel: one group spanning the padded row
    assert _geom(lib, 160, 16, 0, 128) == (0, (256, 256, 1, 64))
    assert _geom(lib, 100, 0, 2, 32)[1] == (128, 32, 4, 0)
    assert _geom(lib, 0, 0, 2, 32)[0] == -1          # bad K
    assert _geom(lib, 64, 0, 7, 32)[0] == -1         # bad mode
    assert _geom(lib, 64, 65, 2, 32)[0] == -1        # S > K


def test_workspace_queries(lib):
    assert lib.sqmp_act_workspace_bytes(16384, 4096, 4096) >= 2 * 4 * 4096 + 4 * 4096
    assert lib.sqmp_pack_workspace_bytes(4096, 11008) >= 2 * 4 * 11008


def test_invalid_arguments_rejected_without_gpu(lib):
    # argument validation happens before any HIP call
    assert lib.sqmp_gemm_fq(None, None, None, None, None, None, 1, 16, 16, 100, 0, 32, 4, 4, None) == -1
    assert lib.sqmp_gemm_f8(None, None, None, None, None, None, None, None, 0, 16, 16, 128, 0, 64, 2, None) == -1
    assert lib.sqmp_quant_act(None, 1, 4, 64, 9, 4, 32, None, 128, None, None, 0, 0, 0, None, None, None, None, 0, None) == -1
    assert lib.sqmp_pack_weight(None, 1, 4, 64, 2, 3, 32, None, 0, None, None, None, None, None, None, None, None, 0, None) == -2


def test_python_surface_mirrors_reference():
    import smoothquant
    from smoothquant import fake_quant, model_size, smooth
    assert smoothquant.__all__ == ["smooth_lm", "quantize_model"]
    sig = inspect.signature(fake_quant.W4A4Linear.__init__)
    assert list(sig.parameters)[1:] == ["in_features", "out_features", "bias", "act_quant",
                                        "quantize_output", "importance", "salient_prop",
                                        "quant_bits", "group_size"]
    sig = inspect.signature(fake_quant.W4A4Linear.from_float)
    assert [(p.name, p.default) for p in sig.parameters.values()] == [
        ("module", inspect._empty), ("weight_quant", "per_channel"), ("act_quant", "per_token"),
        ("quantize_output", False), ("importance", None), ("salient_prop", 0), ("quant_bits", 4),
        ("group_size", 128)]
    assert inspect.signature(fake_quant.quantize_opt).parameters["quantize_bmm_input"].default is True
    assert inspect.signature(fake_quant.quantize_opt).parameters["weight_quant"].default == "per_tensor"
    assert inspect.signature(fake_quant.quantize_llama_like).parameters["quantize_bmm_input"].default is False
    assert inspect.signature(fake_quant.quantize_model).parameters["salient_prop"].default is None
    for name in ("quantize_weight_per_channel_absmax", "quantize_weight_per_tensor_absmax",
                 "quantize_weight_per_group_absmax", "quantize_weight_per_group_absmax_sort",
                 "quantize_activation_per_token_absmax", "quantize_activation_per_tensor_absmax",
                 "quantize_activation_per_group_absmax", "quantize_activation_per_group_absmax_sort",
                 "quantize_mixtral", "quantize_falcon"):
        assert callable(getattr(fake_quant, name))
    assert callable(smooth.smooth_lm) and callable(model_size.get_model_size)


def test_module_host_logic():
    from smoothquant.fake_quant import W4A4Linear
    with pytest.raises(ValueError, match="Invalid act_quant"):
        W4A4Linear(8, 8, act_quant="per_row")
    imp = torch.tensor([0.1, 5.0, 0.3, 5.0, 2.0, 0.0, 1.0, 0.2])
    m = W4A4Linear(8, 4, importance=imp, salient_prop=0.25)
    # ties at the cut-off resolve to the lower channel index (pinned stable rule)
    assert m.salient_indices.tolist() == [1, 3]
    assert W4A4Linear(8, 4, importance=imp, salient_prop=0.01).salient_indices.tolist() == [1]
    assert W4A4Linear(8, 4, importance=None, salient_prop=0.5).salient_indices is None
    r = repr(m)
    assert r.startswith("W4A4Linear(8, 4, bias=True, weight_quant=None, act_quant=per_token")
    # no CPU execution path: forward on a CPU tensor raises instead of falling back
    with pytest.raises((RuntimeError, ValueError)):
        m(torch.zeros(2, 8, dtype=torch.float16))
    with pytest.raises(ValueError, match="Unsupported input shape"):
        m(torch.zeros(1, 1, 2, 8))
    # a kernel name outside the documented set (e.g. the removed "i8") is refused, not
    # silently run on another kernel
    m.kernel = "i8"
    with pytest.raises(ValueError, match="kernel must be one of"):
        m(torch.zeros(2, 8, dtype=torch.float16))
    m.kernel = "auto"
    with pytest.raises(AssertionError):
        W4A4Linear.from_float(torch.nn.Conv1d(2, 2, 1))


def test_quantize_model_dispatch_errors():
    from smoothquant.fake_quant import quantize_model
    with pytest.raises(ValueError, match="Unsupported model type"):
        quantize_model(torch.nn.Linear(4, 4))


def test_model_size_formula():
    from smoothquant.model_size import get_model_size
    lin = torch.nn.Linear(64, 32, bias=False)
    assert get_model_size(lin) == 64 * 32 * 16
    assert get_model_size(lin, data_width=4, salient_prop=0.1, group_size=64) == pytest.approx(
        64 * 32 * ((4 + 20 / 64) * 0.9 + (16 + 20 / 64) * 0.1))


def _c_entries():
    """(name, parameter list, body start) of every extern "C" definition in csrc/."""
    import glob
    out = []
    for f in sorted(glob.glob(os.path.join(ROOT, "smoothquant-mixedprecision_amd", "csrc", "*.hip"))):
        src = open(f).read()
        for m in re.finditer(r'extern "C" [^;{]*?\b(sqmp_[a-z0-9_]+)\s*\(([^)]*)\)\s*\{', src):
            out.append((m.group(1), m.group(2), src[m.end():m.end() + 200]))
    return out


def test_every_launching_entry_runs_on_its_streams_device():
    """Every C entry that takes a stream (i.e. launches work) makes the stream's device
    current first (SQMP_DEVICE_GUARD, sqmp_common.h): the reference's callers place layers on
    several GPUs (accelerate device_map="auto", run_experiments.py:146-148,
    examples/ppl_eval.sh:17-18), so the caller's current device need not be the tensors'."""
    entries = _c_entries()
    declared = set(_declared_functions())
    launching = [(n, body) for n, params, body in entries if re.search(r"void\s*\*\s*stream\b", params)]
    assert len(launching) >= 25
    for n, body in launching:
        first = body.strip().split("\n", 1)[0].strip()
        assert first == "SQMP_DEVICE_GUARD(stream);", f"{n}: first statement is {first!r}"
    # every declared entry that takes a stream is among them
    for n, params, _ in entries:
        if n in declared and "stream" in params:
            assert n in dict(launching), n


def test_lc_lds_budget_in_every_eligibility_check(lib):
    """The lane-contiguous quantizer refuses rows whose LDS image exceeds 150 KiB
    (quant_lc_supported); fqt_eligible, f8_eligible and group_eligible apply the same limit
    (ops.lc_lds_ok), so such a layer takes another path instead of raising EUNSUPPORTED.
    K = 16384, G = 128: half salient fits, two thirds does not."""
    from types import SimpleNamespace
    from smoothquant import ops

    def pw(S):
        g = [ctypes.c_int() for _ in range(4)]
        assert lib.sqmp_weight_geometry(16384, S, 2, 128, *[ctypes.byref(v) for v in g]) == 0
        Kp, Gw, ngw, S_pad = (v.value for v in g)
        return SimpleNamespace(K=16384, S=S, Kp=Kp, S_pad=S_pad, Gw=Gw, ngw=ngw, N=4096,
                               n_bits=4, dense=None, dtype=torch.float16)

    ok, big = pw(8192), pw(11000)
    assert ops.lc_lds_ok(ok.Kp, ok.S_pad) and not ops.lc_lds_ok(big.Kp, big.S_pad)
    # the boundary itself: 4 * lc_lds_words(P, S_pad, 1) <= 150 KiB
    P = 16384
    S_max = (150 * 1024 // 4 - P - 8 - 2 * (P // 64)) // 2
    assert ops.lc_lds_ok(P, S_max) and not ops.lc_lds_ok(P, S_max + 1)
    assert ops.fqt_eligible(ok, "per_group", 4, 128, 16384, force=True)
    assert not ops.fqt_eligible(big, "per_group", 4, 128, 16384, force=True)
    assert ops.f8_eligible(ok, "per_token", 4) and not ops.f8_eligible(big, "per_token", 4)
