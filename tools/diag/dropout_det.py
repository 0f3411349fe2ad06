"""Diagnostic: weight differences after 40 dropout-0.2 steps — eager vs eager
(same seed base) and eager vs FeederGraph — to tell atomic-order noise from a
mask mismatch."""
import copy
import sys

import torch

sys.path[:0] = ["real-time-recommendation-system-with-feature-store_amd", "."]
from rtrec_amd.data.movielens import synthetic_movielens  # noqa: E402
from rtrec_amd.training.datasets.movielens import DeviceFeeder  # noqa: E402
from rtrec_amd.training.fused_step import FeederGraph, FusedTrainStep  # noqa: E402
from rtrec_amd.training.utils import create_two_tower_model_for_training  # noqa: E402

dev = torch.device("cuda:0")
data = synthetic_movielens(seed=0)
for p in (0.0, 0.2):
    torch.manual_seed(7)
    cfg = {"embedding_dim": 64, "hidden_layers": [256, 128], "dropout_rate": p, "temperature": 0.05}
    m0 = create_two_tower_model_for_training(3, 20, cfg)
    ms = [copy.deepcopy(m0).to(dev) for _ in range(3)]
    fs = [DeviceFeeder(data.train_interactions, data.users, data.movies, num_negatives=16, batch_size=256,
                       device=dev, seed=5) for _ in range(3)]
    ss = [FusedTrainStep(m, dropout_seed=1234) for m in ms]
    losses = []
    for j in range(2):
        ls = []
        for i, b in enumerate(fs[j]):
            if i == 40:
                break
            ls.append(float(ss[j](b["user_table"], b["item_table"], b["item_table"], user_ids=b["user_ids"],
                                  pos_ids=b["pos_ids"], neg_ids=b["neg_ids"])[0].item()))
        losses.append(ls)
    g = FeederGraph(ss[2], fs[2]).run_epoch(max_batches=40).cpu().tolist()
    losses.append(g)
    init = copy.deepcopy(m0).to(dev).state_dict()
    for name, (a, b_) in {"eager-eager": (0, 1), "eager-graph": (0, 2)}.items():
        worst = max(((ka, float((va.float() - vb.float()).abs().max())) for (ka, va), vb in
                     zip(ms[a].state_dict().items(), ms[b_].state_dict().values()) if va.numel()), key=lambda t: t[1])
        lrel = max(abs(x - y) / abs(x) for x, y in zip(losses[a], losses[b_]))
        print(f"p={p} {name}: max weight diff {worst}, max loss rel {lrel:.3g}")
    move = max(float((v.float() - init[k].float()).abs().max()) for k, v in ms[0].state_dict().items()
               if v.dtype.is_floating_point)
    print(f"p={p} max weight movement {move:.4g}")
