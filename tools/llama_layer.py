"""bench.py's llama_layer line alone (Llama-2-7B decoder-layer linears at 2048 tokens, W4A4 vs
fp16 F.linear) -- a target for rocprofv3 --kernel-trace --stats.  python tools/llama_layer.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

print(json.dumps(bench.llama_layer(torch.device("cuda"))))
