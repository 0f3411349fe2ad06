"""C1 epoch timing (bench.c1_epoch: emb 64, batch 256, 16 negatives, one full
epoch through the feeder graph) printed as one JSON line; for env A/Bs."""
import json
import os
import sys

import torch

sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."),
                os.path.join(os.path.dirname(__file__), "..", "real-time-recommendation-system-with-feature-store_amd")]
import bench  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
runs = [bench.c1_epoch(dev)["ms_per_batch"] for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 2)]
print(json.dumps({"env_RT_DZ_KSPLIT": os.environ.get("RT_DZ_KSPLIT", "auto"), "ms_per_batch": runs}))
