"""The headline C2 step at exactly the benchmarked shape, against the oracle.

bench.py times FusedTrainStep on ``bench.c2_setup``: ML-1M-shaped feature
tables resident on the device, B=1024 users, N=16 negatives (17,408 item-tower
rows per step through the fused-gather id path, positives and negatives
adjacent in one id buffer), emb 128, hidden [256,128], tau 0.05, Adam(1e-3,
wd 1e-5) + clip 1.0, replayed as a hipGraph. Here the same setup runs with
dropout 0 (the dropout RNG is the only term the oracle cannot reproduce; its
mask contract is tests/test_gpu_dropout.py) for 3 steps, eagerly and as graph
replays, and is compared step by step with oracle/two_tower.train_step — the
restatement of TwoTowerTrainer.train_epoch (src/training/trainers/
two_tower.py:98-146) pinned by tests/golden/train_step_c2.npz. This is the
shape at which the dW split plan (cap 64 splits for 8-tile layers, ~1024
blocks) and the merged pos/neg item chain engage.

Bars: loss (mixed, explicit, in-batch) within 1e-4 relative (north_star);
parameters as in the B=64 golden test (Adam moves each weight by ~lr per
step, so elements whose gradient is ~0 may differ by up to one lr per step);
BN running statistics within 1e-4 relative."""
import copy
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

REPO = Path(__file__).resolve().parent.parent
STEPS = 3
RTOL = 1e-4


@pytest.fixture(scope="module")
def c2(device):
    if str(REPO) not in sys.path:
        sys.path.insert(0, str(REPO))
    import bench
    model, (ut, mt), batches, host = bench.c2_setup(device, 0, STEPS, dropout=0.0)
    uf, mf, bu, bp, bn = host
    return bench, model, ut, mt, batches, (uf, mf, bu, bp, bn)


@pytest.fixture(scope="module")
def oracle_run(c2):
    """STEPS oracle steps from the model's initial state: per-step losses and
    the post-step tower states."""
    from oracle import two_tower as orc
    _, model, _, _, _, (uf, mf, bu, bp, bn) = c2
    us = {k: v.detach().cpu().clone() for k, v in model.user_tower.state_dict().items()}
    its = {k: v.detach().cpu().clone() for k, v in model.item_tower.state_dict().items()}
    biases = {"user_bias": model.user_bias.detach().cpu().clone(), "item_bias": model.item_bias.detach().cpu().clone()}
    opt, out = {}, []
    for i in range(STEPS):
        u = torch.from_numpy(uf[bu[i]])
        p = torch.from_numpy(mf[bp[i]])
        n = torch.from_numpy(mf[bn[i]]).view(1024, 16, 20)
        r = orc.train_step(us, its, biases, opt, u, p, n, temperature=0.05, lr=1e-3, weight_decay=1e-5)
        out.append((r, {k: v.detach().clone() for k, v in us.items()}, {k: v.detach().clone() for k, v in its.items()},
                    {k: v.detach().clone() for k, v in biases.items()}))
    return out


def _compare(step_i, loss_dev, model, ref):
    r, us, its, biases = ref
    lb = loss_dev.detach().cpu().numpy()
    np.testing.assert_allclose(lb, [r["loss"], r["explicit"], r["in_batch"]], rtol=RTOL,
                               err_msg=f"step {step_i} loss (mixed, explicit, in-batch)")
    for tname, tower, ref_state in (("user", model.user_tower, us), ("item", model.item_tower, its)):
        for k, v in tower.state_dict().items():
            got = v.detach().cpu().numpy()
            want = ref_state[k].numpy()
            if "num_batches" in k:
                assert int(got) == int(want), (step_i, tname, k)
                continue
            if "running" in k:
                np.testing.assert_allclose(got, want, rtol=RTOL, atol=1e-6, err_msg=f"step {step_i} {tname}.{k}")
                continue
            diff = np.abs(got - want)
            close = np.mean(diff <= 1e-5 + 1e-4 * np.abs(want))
            assert close > 0.99, (step_i, tname, k, close, diff.max())
            assert diff.max() <= 1.05e-3 * (step_i + 1) + 1e-5, (step_i, tname, k, diff.max())
    for k in ("user_bias", "item_bias"):
        got = float(getattr(model, k).detach().cpu())
        assert abs(got - float(biases[k])) <= 1.05e-3 * (step_i + 1) + 1e-6, (step_i, k)


def test_c2_fullsize_eager_vs_oracle(c2, oracle_run):
    from rtrec_amd.training.fused_step import FusedTrainStep
    _, model0, ut, mt, batches, _ = c2
    model = copy.deepcopy(model0).to(ut.device)
    step = FusedTrainStep(model, lr=1e-3, weight_decay=1e-5, max_norm=1.0)
    for i in range(STEPS):
        bu, bp, bn = batches[i]
        assert bn.data_ptr() == bp.data_ptr() + bp.numel() * 8  # the bench's adjacent pos/neg id layout
        loss = step(ut, mt, mt, user_ids=bu, pos_ids=bp, neg_ids=bn)
        torch.cuda.synchronize()
        _compare(i, loss, model, oracle_run[i])


def test_c2_fullsize_graph_replay_vs_oracle(c2, oracle_run):
    """The bench's timed form: one hipGraph captured over static id buffers
    (warmup restored), new ids copied in before every replay."""
    from rtrec_amd.training.fused_step import FusedTrainStep
    _, model0, ut, mt, batches, _ = c2
    model = copy.deepcopy(model0).to(ut.device)
    step = FusedTrainStep(model, lr=1e-3, weight_decay=1e-5, max_norm=1.0)
    b0 = batches[0]
    st_pn = torch.cat([b0[1].reshape(-1), b0[2].reshape(-1)])
    st = (b0[0].clone(), st_pn[:b0[1].numel()].view(b0[1].shape), st_pn[b0[1].numel():].view(b0[2].shape))
    step.capture(ut, mt, mt, user_ids=st[0], pos_ids=st[1], neg_ids=st[2], warmup=1)
    for i in range(STEPS):
        for dst, src in zip(st, batches[i]):
            dst.copy_(src)
        loss = step.replay()
        torch.cuda.synchronize()
        _compare(i, loss, model, oracle_run[i])
