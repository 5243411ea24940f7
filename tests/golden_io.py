"""Loader for tests/golden/fake_quant_golden.npz (plain arrays; no pickle)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                      "fake_quant_golden.npz")


def _bf16_to_f32(a: np.ndarray) -> np.ndarray:
    return (a.astype(np.uint32) << 16).view(np.float32)


class Golden:
    def __init__(self, path=GOLDEN):
        self.z = np.load(path, allow_pickle=False)
        self.meta = json.loads(bytes(self.z["meta_json"]).decode())

    def arr(self, key, dt):
        a = self.z[key]
        if dt == "bf16":
            return _bf16_to_f32(a)
        return a

    def has(self, key):
        return key in self.z.files
