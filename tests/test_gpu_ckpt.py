""".pth interop: checkpoints WRITTEN BY THE REFERENCE
(tests/golden/ckpt_ref_model.pth from TwoTowerModel.save_model,
src/models/two_tower.py:516-529, and ckpt_ref_trainer.pth from
TwoTowerTrainer.save_checkpoint, src/training/trainers/two_tower.py:190-215,
both produced by tools/make_goldens.py --only r2) load here with
weights_only=True and reproduce the reference's embeddings; the trainer
checkpoint resumes (Adam moments + step) and the next fused step matches the
step the reference's own optimizer took after writing it."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

CFG = {"embedding_dim": 64, "hidden_layers": [128, 64], "dropout_rate": 0.0, "temperature": 0.05}


def _embed(m, g, dev):
    m.eval()
    with torch.no_grad():
        ue = m.get_user_embeddings({"numerical": torch.from_numpy(g["q_user"]).to(dev), "categorical": {}})
        ie = m.get_item_embeddings({"numerical": torch.from_numpy(g["q_item"]).to(dev), "categorical": {}})
    return ue.cpu().numpy(), ie.cpu().numpy()


def test_load_reference_save_model(device, golden):
    from conftest import GOLDEN
    from rtrec_amd.training.utils import create_two_tower_model_for_training
    g = golden("ckpt_ref_expect")
    m = create_two_tower_model_for_training(3, 20, CFG)
    m.load_model(str(GOLDEN / "ckpt_ref_model.pth"))
    m.to(device)
    ue, ie = _embed(m, g, device)
    np.testing.assert_allclose(ue, g["user_emb"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(ie, g["item_emb"], rtol=1e-5, atol=1e-6)
    assert m.temperature == pytest.approx(0.05)


def test_evaluate_model_load_model_infers_architecture(device, golden):
    from conftest import GOLDEN
    from rtrec_amd.evaluation import load_model
    g = golden("ckpt_ref_expect")
    m = load_model(str(GOLDEN / "ckpt_ref_trainer.pth"), user_dim=3, item_dim=20, device="cuda")
    assert [m.user_tower.mlp[0].out_features, m.user_tower.mlp[4].out_features] == [128, 64]
    ue, ie = _embed(m, g, device)
    np.testing.assert_allclose(ue, g["user_emb"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(ie, g["item_emb"], rtol=1e-5, atol=1e-6)


def test_trainer_resumes_reference_checkpoint(device, golden, tmp_path):
    from conftest import GOLDEN
    from rtrec_amd.training.trainers.two_tower import TwoTowerTrainer
    from rtrec_amd.training.utils import create_two_tower_model_for_training
    g = golden("ckpt_ref_expect")
    m = create_two_tower_model_for_training(3, 20, CFG)
    tr = TwoTowerTrainer(m, [], [], {"learning_rate": 1e-3, "weight_decay": 1e-5, "checkpoint_dir": str(tmp_path)},
                         device="cuda")
    epoch = tr.load_checkpoint(GOLDEN / "ckpt_ref_trainer.pth")
    assert epoch == 1
    np.testing.assert_allclose(tr.train_losses, g["losses"][:1], rtol=1e-12)
    assert int(tr.step.step_dev.item()) == 1
    # the loaded Adam state is the reference optimizer's, bit for bit, in its
    # parameter order (a swapped mapping or a biased step count fails here)
    ref_ck = torch.load(GOLDEN / "ckpt_ref_trainer.pth", map_location="cpu", weights_only=True)
    mine = tr.step.optimizer_state_dict()["state"]
    assert set(mine) == set(ref_ck["optimizer_state"]["state"])
    for i, st in ref_ck["optimizer_state"]["state"].items():
        assert torch.equal(mine[i]["exp_avg"].cpu(), st["exp_avg"]), i
        assert torch.equal(mine[i]["exp_avg_sq"].cpu(), st["exp_avg_sq"]), i
        assert float(mine[i]["step"]) == float(st["step"])
    batch = {k[3:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("b1_")}
    tr.train_loader = [batch]
    loss = tr.train_epoch(2)
    np.testing.assert_allclose(loss, g["losses"][1], rtol=1e-4)
    for tname, tower in (("user", m.user_tower), ("item", m.item_tower)):
        for k, v in tower.state_dict().items():
            ref = g[f"after_{tname}/{k}"]
            got = v.detach().cpu().numpy()
            if "num_batches" in k:
                assert int(got) == int(ref), k
                continue
            diff = np.abs(got - ref)
            # second Adam step from identical moments: ~lr-sized moves, tight elsewhere
            assert np.mean(diff <= 1e-5 + 1e-4 * np.abs(ref)) > 0.995, (k, diff.max())
            assert diff.max() <= 1.1e-3, (k, diff.max())
    # the moments after that step against the reference optimizer's own
    # (tests/golden/ckpt_ref_moments.npz): tight, since both start from the
    # same state and differ only by the fp32 gradient rounding
    mo = golden("ckpt_ref_moments")
    after = tr.step.optimizer_state_dict()["state"]
    for i, st in after.items():
        assert float(st["step"]) == float(mo[f"step/{i}"]) == 2.0
        for name in ("exp_avg", "exp_avg_sq"):
            ref = mo[f"{name}/{i}"]
            np.testing.assert_allclose(st[name].cpu().numpy(), ref, rtol=1e-4, atol=1e-6 * float(np.abs(ref).max() + 1e-30),
                                       err_msg=f"{name}/{i}")
    # and what we write reads back in the same layout (our save -> our resume)
    tr.save_checkpoint(2, is_best=True)
    ck = torch.load(tmp_path / "two_tower_best.pth", map_location="cpu", weights_only=True)
    assert set(ck) == set(ref_ck)
    assert set(ck["optimizer_state"]["state"]) == set(ref_ck["optimizer_state"]["state"])
    assert ck["epoch"] == 2
