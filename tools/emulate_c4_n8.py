#!/usr/bin/env python3
"""bench.topk_c4_n8_emulated on its own (the per-rank C4 work at N = 8 on one GPU)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "real-time-recommendation-system-with-feature-store_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

from rtrec_amd import native  # noqa: E402

native.lib()
print(json.dumps(bench.topk_c4_n8_emulated(torch.device("cuda:0"))), flush=True)
