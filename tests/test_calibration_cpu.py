"""Calibration statistics (smoothquant.calibration) against the reference-generated
tiny-model fixtures: the mean|x| importance features and the channel absmax act scales
of the unquantized models, bit-exact, plus the calibration-block builder and the
Evaluator formula."""
import copy

import pytest
import torch

from model_cases import ModelGolden, build_model, cal_blocks
from smoothquant.calibration import get_act_scales, get_calib_dataset, get_calib_feat
from smoothquant.ppl import Evaluator

MG = ModelGolden()


class BlockTokenizer:
    """Maps the text "<i>" to calibration block i (for the json-dataset entry points)."""

    def __init__(self, blocks):
        self.blocks = blocks

    class _Out:
        def __init__(self, ids):
            self.input_ids = ids

    def __call__(self, text, return_tensors=None, max_length=None, truncation=False):
        ids = self.blocks[int(text)]
        if truncation and max_length:
            ids = ids[:, :max_length]
        return self._Out(ids)

    def encode(self, text):
        return [int(c) for c in text.split()] if text.strip() else []


@pytest.mark.parametrize("case", MG.cases(), ids=[c["key"] for c in MG.cases()])
def test_calibration_matches_reference_fixtures(case):
    model = build_model(case)
    blocks = cal_blocks(case)
    if case["alpha"] is not None:
        tok = BlockTokenizer(blocks)
        sc = get_act_scales(copy.deepcopy(model), tok, [{"text": str(i)} for i in range(len(blocks))],
                            num_samples=len(blocks), seq_len=512)
        want = MG.scales(case["key"])
        assert set(sc) == set(want)
        for k in want:
            assert torch.equal(sc[k], want[k]), k
        from smoothquant.smooth import smooth_lm
        smooth_lm(model, want, case["alpha"])
    want = MG.feat(case["key"])
    if want is not None:
        feat = get_calib_feat(model, None, samples=blocks, device="cpu")
        assert set(feat) == set(want)
        for k in want:
            assert len(feat[k]) == len(want[k])
            for a, b in zip(feat[k], want[k]):
                assert torch.equal(a, b), k


def test_calib_dataset_blocks():
    """run_experiments.py:30-53: shuffle(seed=42), skip lines longer than block_size and
    empty lines, stop after n_samples kept lines, concatenate, cut block_size blocks."""
    from datasets import Dataset
    tok = BlockTokenizer([])
    rows = [{"text": " ".join(str(100 * i + j) for j in range(n))}
            for i, n in enumerate([3, 0, 5, 9, 2, 4, 7, 1])]
    n_samples, B = 4, 5
    blocks = get_calib_dataset(tok, n_samples=n_samples, block_size=B, dataset=rows)
    kept = []
    for r in Dataset.from_list(rows).shuffle(seed=42):
        ids = tok.encode(r["text"].strip())
        if 0 < len(ids) <= B:
            kept.append(ids)
        if len(kept) == n_samples:
            break
    flat = [t for ids in kept for t in ids]
    assert len(blocks) == len(flat) // B
    for i, b in enumerate(blocks):
        assert b.shape == (1, B) and b[0].tolist() == flat[i * B:(i + 1) * B]


def test_evaluator_formula():
    case = MG.cases()[0]
    model = build_model(case)
    ids = torch.from_numpy(MG.arr(case["key"], "ev").copy())
    B = case["eval_window"]
    ev = Evaluator(None, None, "cpu", n_samples=ids.size(1) // B, batch_size=B, input_ids=ids)
    ppl = float(ev.evaluate(model))
    # restated: exp(mean over windows of the mean CE)
    ces = []
    with torch.no_grad():
        for i in range(ids.size(1) // B):
            b = ids[:, i * B:(i + 1) * B]
            lg = model(b).logits[:, :-1].float()
            ces.append(torch.nn.functional.cross_entropy(lg.reshape(-1, lg.size(-1)), b[:, 1:].reshape(-1)))
    assert abs(ppl - float(torch.exp(torch.stack(ces).mean()))) <= 1e-3 * ppl
    assert ev.last_tokens_per_s and ev.last_tokens_per_s > 0


def test_evaluator_short_last_window_scales_by_batch_size():
    """n_samples beyond the full windows: the reference scales every window's mean CE by
    self.batch_size, the short last one too (run_experiments.py:116-123)."""
    case = MG.cases()[0]
    model = build_model(case)
    ids = torch.from_numpy(MG.arr(case["key"], "ev").copy())
    B = case["eval_window"]
    n_full = ids.size(1) // B - 1
    assert n_full >= 1
    ids = ids[:, : n_full * B + B // 2]          # one half window at the end
    ev = Evaluator(None, None, "cpu", n_samples=n_full + 1, batch_size=B, input_ids=ids)
    ppl = float(ev.evaluate(model))
    nlls = []
    with torch.no_grad():
        for i in range(n_full + 1):
            b = ids[:, i * B:(i + 1) * B]
            lg = model(b).logits[:, :-1].float()
            ce = torch.nn.functional.cross_entropy(lg.reshape(-1, lg.size(-1)), b[:, 1:].reshape(-1))
            nlls.append(ce.float() * B)
    want = float(torch.exp(torch.stack(nlls).sum() / ((n_full + 1) * B)))
    assert abs(ppl - want) <= 1e-4 * want


def test_evaluator_default_window_count_is_per_2048_tokens():
    """n_samples falsy: the reference evaluates dataset.size(1) // 2048 windows of batch_size
    tokens (run_experiments.py:103), not size // batch_size."""
    case = MG.cases()[0]
    model = build_model(case)
    base = torch.from_numpy(MG.arr(case["key"], "ev").copy())
    ids = base.repeat(1, 4196 // base.size(1) + 1)[:, :4196]   # 2 x 2048 + 100 tokens
    B = 256
    ev = Evaluator(None, None, "cpu", n_samples=None, batch_size=B, input_ids=ids)
    wins = ev.windows()
    assert len(wins) == 2 and all(w.shape == (1, B) for w in wins)
    assert torch.equal(wins[1], ids[:, B:2 * B])
    ppl = float(ev.evaluate(model))
    nlls = []
    with torch.no_grad():
        for w in wins:
            lg = model(w).logits[:, :-1].float()
            ce = torch.nn.functional.cross_entropy(lg.reshape(-1, lg.size(-1)), w[:, 1:].reshape(-1))
            nlls.append(ce.float() * B)
    want = float(torch.exp(torch.stack(nlls).sum() / (2 * B)))
    assert abs(ppl - want) <= 1e-4 * want
