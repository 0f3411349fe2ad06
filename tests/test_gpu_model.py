"""GPU parity of the two-tower model surface (fused MLP / loss / optimiser
kernels) against golden vectors produced by the reference, plus the
reference's own behavioural pins (tests/test_two_tower_model.py:29-361)
replayed on the MI355X path."""
import tempfile
from pathlib import Path

import numpy as np
import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu

RTOL = 1e-4  # north_star: loss/scores within 1e-4 relative


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from rtrec_amd import native
    native.lib()
    return torch.device("cuda:0")


def _mods():
    from rtrec_amd.models.two_tower import ItemTower, TwoTowerModel, UserTower, create_two_tower_model
    return UserTower, ItemTower, TwoTowerModel, create_two_tower_model


def _tower_for(name):
    UserTower, ItemTower, _, _ = _mods()
    if name == "tower_user_c2":
        return UserTower(3, 128, [256, 128], dropout_rate=0.0)
    if name == "tower_item_c2":
        return ItemTower(20, 128, [256, 128], dropout_rate=0.0, use_content_embedding=False)
    if name == "tower_user_cat":
        return UserTower(10, 32, [64, 32], dropout_rate=0.0, categorical_features={"category": 10, "subcategory": 5})
    if name == "tower_item_content":
        return ItemTower(15, 32, [64, 32], dropout_rate=0.0, use_content_embedding=True, content_embedding_dim=768)
    act = name.split("tower_act_")[1]
    return UserTower(10, 32, [64, 48], dropout_rate=0.0, activation=act)


def _load_state(module, g, prefix="state"):
    sd = {k[len(prefix) + 1:]: torch.from_numpy(np.array(v)) for k, v in g.items() if k.startswith(prefix + "/")}
    module.load_state_dict(sd)


TOWER_CASES = ["tower_user_c2", "tower_item_c2", "tower_user_cat", "tower_item_content",
               "tower_act_gelu", "tower_act_leaky_relu", "tower_act_tanh", "tower_act_sigmoid"]


@pytest.mark.parametrize("name", TOWER_CASES)
def test_tower_golden_eval_train_backward(dev, golden, name):
    g = golden(name)
    t = _tower_for(name)
    _load_state(t, g)
    t.to(dev)
    x = torch.from_numpy(g["x"]).to(dev)
    cat = {k[4:]: torch.from_numpy(v).to(dev) for k, v in g.items() if k.startswith("cat/")} or None
    content = torch.from_numpy(g["content"]).to(dev) if "content" in g else None
    args = (x, cat, content) if content is not None else (x, cat)
    t.eval()
    with torch.no_grad():
        y = t(*args)
    np.testing.assert_allclose(y.cpu().numpy(), g["out_eval"], rtol=RTOL, atol=2e-6)
    t.train()
    xg = x.clone().requires_grad_(True)
    args = (xg, cat, content) if content is not None else (xg, cat)
    y = t(*args)
    np.testing.assert_allclose(y.detach().cpu().numpy(), g["out_train"], rtol=RTOL, atol=2e-6)
    (y * torch.from_numpy(g["r"]).to(dev)).sum().backward()
    np.testing.assert_allclose(xg.grad.cpu().numpy(), g["grad_x"], rtol=1e-3, atol=1e-5)
    for k, p in t.named_parameters():
        ref = g.get(f"grad/{k}")
        if ref is None:
            continue
        # fp32 reductions in a different order: tolerance relative to the gradient's scale
        np.testing.assert_allclose(p.grad.cpu().numpy(), ref, rtol=1e-3, atol=1e-4 * np.abs(ref).max() + 1e-7,
                                   err_msg=k)
    sd = t.state_dict()
    for k, v in g.items():
        if k.startswith("post/"):
            np.testing.assert_allclose(sd[k[5:]].cpu().numpy(), v, rtol=1e-5, atol=1e-6, err_msg=k)


@pytest.mark.parametrize("b,d", [(8, 64), (8, 128), (256, 64), (256, 128), (1024, 128)])
def test_in_batch_loss_golden(dev, golden, b, d):
    _, _, TwoTowerModel, _ = _mods()
    UserTower, ItemTower, _, _ = _mods()
    g = golden(f"loss_inbatch_B{b}_D{d}")
    m = TwoTowerModel(UserTower(4, 8, [8]), ItemTower(4, 8, [8], use_content_embedding=False),
                      temperature=float(g["tau"])).to(dev)
    u = torch.from_numpy(g["u"]).to(dev).requires_grad_(True)
    i = torch.from_numpy(g["i"]).to(dev).requires_grad_(True)
    loss = m.in_batch_negative_loss(u, i)
    loss.backward()
    np.testing.assert_allclose(loss.item(), g["loss"], rtol=RTOL)
    np.testing.assert_allclose(u.grad.cpu().numpy(), g["grad_u"], rtol=1e-3, atol=1e-6)
    np.testing.assert_allclose(i.grad.cpu().numpy(), g["grad_i"], rtol=1e-3, atol=1e-6)


def test_contrastive_loss_golden(dev, golden):
    UserTower, ItemTower, TwoTowerModel, _ = _mods()
    g = golden("loss_contrastive")
    m = TwoTowerModel(UserTower(4, 8, [8]), ItemTower(4, 8, [8], use_content_embedding=False),
                      temperature=float(g["tau"])).to(dev)
    with torch.no_grad():
        m.user_bias.fill_(float(g["user_bias"]))
        m.item_bias.fill_(float(g["item_bias"]))
    u = torch.from_numpy(g["u"]).to(dev).requires_grad_(True)
    p = torch.from_numpy(g["p"]).to(dev).requires_grad_(True)
    n = torch.from_numpy(g["n"]).to(dev).requires_grad_(True)
    loss = m.contrastive_loss(u, p, n)
    loss.backward()
    np.testing.assert_allclose(loss.item(), g["loss"], rtol=RTOL)
    for t, k in [(u, "grad_u"), (p, "grad_p"), (n, "grad_n")]:
        np.testing.assert_allclose(t.grad.cpu().numpy(), g[k], rtol=1e-3, atol=1e-6, err_msg=k)
    np.testing.assert_allclose(m.user_bias.grad.cpu().numpy(), g["grad_user_bias"], rtol=1e-4, atol=1e-7)
    np.testing.assert_allclose(m.item_bias.grad.cpu().numpy(), g["grad_item_bias"], rtol=1e-4, atol=1e-7)


def test_similarity_golden(dev, golden):
    UserTower, ItemTower, TwoTowerModel, _ = _mods()
    g = golden("similarity")
    m = TwoTowerModel(UserTower(4, 8, [8]), ItemTower(4, 8, [8], use_content_embedding=False),
                      temperature=float(g["tau"])).to(dev)
    with torch.no_grad():
        m.user_bias.fill_(float(g["user_bias"]))
        m.item_bias.fill_(float(g["item_bias"]))
    s = m.compute_similarity(torch.from_numpy(g["u"]).to(dev), torch.from_numpy(g["i"]).to(dev))
    np.testing.assert_allclose(s.detach().cpu().numpy(), g["sim"], rtol=RTOL, atol=1e-5)


def _flat_state(g, prefix):
    return {k[len(prefix) + 1:]: torch.from_numpy(np.array(v)) for k, v in g.items() if k.startswith(prefix + "/")}


def test_fused_train_step_golden(dev, golden):
    """Two TwoTowerTrainer.train_epoch steps of the reference (C2 architecture,
    dropout 0): loss within 1e-4 rel, parameters after Adam close."""
    from rtrec_amd.training.fused_step import FusedTrainStep
    from rtrec_amd.training.utils import create_two_tower_model_for_training
    g = golden("train_step_c2")
    model = create_two_tower_model_for_training(3, 20, {"embedding_dim": 128, "hidden_layers": [256, 128],
                                                        "dropout_rate": 0.0, "temperature": 0.05})
    model.user_tower.load_state_dict(_flat_state(g, "user"))
    model.item_tower.load_state_dict(_flat_state(g, "item"))
    model.to(dev)
    step = FusedTrainStep(model, lr=1e-3, weight_decay=1e-5)
    losses = []
    for j, pre in enumerate(["mid", "final"]):
        lb = step(torch.from_numpy(g[f"b{j}_user_features"]).to(dev),
                  torch.from_numpy(g[f"b{j}_pos_item_features"]).to(dev),
                  torch.from_numpy(g[f"b{j}_neg_item_features"]).to(dev))
        losses.append(float(lb[0].item()))
        for tname, tower in (("user", model.user_tower), ("item", model.item_tower)):
            for k, v in tower.state_dict().items():
                ref = g[f"{pre}_{tname}/{k}"]
                got = v.detach().cpu().numpy()
                if "num_batches" in k:
                    assert int(got) == int(ref), k
                    continue
                # Adam's first steps move each weight by ~lr·sign(g): tolerate 2 lr-steps
                # on elements whose gradient is ~0, require closeness everywhere else
                diff = np.abs(got - ref)
                assert np.mean(diff <= 1e-5 + 1e-4 * np.abs(ref)) > 0.995, (k, diff.max())
                assert diff.max() <= 2.1e-3, (k, diff.max())
    np.testing.assert_allclose(losses, g["losses"], rtol=RTOL)


def test_fused_train_step_mixed_dw_prologues(dev):
    """Tower pairs whose paired layers differ in in_features % 4: the user
    tower's last Linear (in 130) recomputes its input in the dW launch while the
    item tower's (in 128) reads the forward's staged rows, so the joint dW launch
    splits into two single-set launches. Their row-split plans must match the
    partial buffers the caller sized (rt_linear_bwd_dw_splits) and the dz fusion
    must not add dbias twice. Two steps against oracle.train_step."""
    from oracle import two_tower as orc
    from rtrec_amd.models.two_tower import ItemTower, TwoTowerModel, UserTower
    from rtrec_amd.training.fused_step import FusedTrainStep
    torch.manual_seed(5)
    model = TwoTowerModel(UserTower(3, 64, [256, 130], dropout_rate=0.0),
                          ItemTower(20, 64, [256, 128], dropout_rate=0.0, use_content_embedding=False),
                          temperature=0.05)
    us = {k: v.detach().clone() for k, v in model.user_tower.state_dict().items()}
    its = {k: v.detach().clone() for k, v in model.item_tower.state_dict().items()}
    biases = {"user_bias": model.user_bias.detach().clone(), "item_bias": model.item_bias.detach().clone()}
    model.to(dev)
    step = FusedTrainStep(model, lr=1e-3, weight_decay=1e-5)
    g = torch.Generator().manual_seed(9)
    opt = {}
    for _ in range(2):
        u = torch.randn(256, 3, generator=g)
        p = torch.randn(256, 20, generator=g)
        n = torch.randn(256, 4, 20, generator=g)
        r = orc.train_step(us, its, biases, opt, u, p, n, temperature=0.05, lr=1e-3, weight_decay=1e-5)
        lb = step(u.to(dev), p.to(dev), n.to(dev))
        np.testing.assert_allclose(float(lb[0].item()), r["loss"], rtol=RTOL)
    for tname, tower, ref_sd in (("user", model.user_tower, us), ("item", model.item_tower, its)):
        for k, v in tower.state_dict().items():
            ref = ref_sd[k].detach().numpy()
            got = v.detach().cpu().numpy()
            if "num_batches" in k:
                assert int(got) == int(ref), k
                continue
            diff = np.abs(got - ref)
            assert np.mean(diff <= 1e-5 + 1e-4 * np.abs(ref)) > 0.995, (tname, k, diff.max())
            assert diff.max() <= 2.1e-3, (tname, k, diff.max())


# ---------------------------------------------------------------------------
# reference behavioural tests (tests/test_two_tower_model.py) on the GPU path
# ---------------------------------------------------------------------------
def test_user_tower_shapes_norms_batches(dev):
    UserTower, _, _, _ = _mods()
    t = UserTower(input_dim=10, embedding_dim=32, hidden_layers=[64, 32], dropout_rate=0.1).to(dev)
    out = t(torch.randn(8, 10, device=dev))
    assert out.shape == (8, 32)
    assert torch.allclose(out.norm(dim=1), torch.ones(8, device=dev), atol=1e-5)
    t.eval()
    for bsz in [1, 4, 16, 64]:
        assert t(torch.randn(bsz, 10, device=dev)).shape == (bsz, 32)


def test_batchnorm_train_single_row_raises(dev):
    UserTower, _, _, _ = _mods()
    t = UserTower(10, 32, [64, 32]).to(dev)
    with pytest.raises(ValueError, match="more than 1 value"):
        t(torch.randn(1, 10, device=dev))


def test_categorical_and_gradient_flow(dev):
    UserTower, _, _, _ = _mods()
    t = UserTower(10, 32, [64, 32], categorical_features={"category": 10, "subcategory": 5}).to(dev)
    cat = {"category": torch.randint(0, 10, (8,), device=dev), "subcategory": torch.randint(0, 5, (8,), device=dev)}
    assert t(torch.randn(8, 10, device=dev), cat).shape == (8, 32)
    with pytest.raises(RuntimeError, match="cannot be multiplied"):
        t(torch.randn(8, 10, device=dev))  # missing categorical inputs: width mismatch, like F.linear
    t2 = UserTower(10, 32, [64, 32], dropout_rate=0.1).to(dev)
    x = torch.randn(4, 10, device=dev, requires_grad=True)
    t2(x).sum().backward()
    assert x.grad is not None and not torch.all(x.grad == 0)
    # embedding gradients reach the tables (padding row 0 excluded)
    xn = torch.randn(8, 10, device=dev, requires_grad=True)
    ids = torch.tensor([0, 1, 2, 3, 0, 5, 6, 7], device=dev)
    t(xn, {"category": ids, "subcategory": ids % 5}).sum().backward()
    ge = t.embeddings["category"].weight.grad
    assert torch.all(ge[0] == 0) and ge[1].abs().sum() > 0 and torch.all(ge[8:] == 0)


def test_item_tower_content(dev):
    _, ItemTower, _, _ = _mods()
    t = ItemTower(15, 32, [64, 32], use_content_embedding=True, content_embedding_dim=768).to(dev)
    out = t(torch.randn(8, 15, device=dev), content_embeddings=torch.randn(8, 768, device=dev))
    assert out.shape == (8, 32)


def _small_model(dev):
    UserTower, ItemTower, TwoTowerModel, _ = _mods()
    return TwoTowerModel(UserTower(10, 32, [64, 32]), ItemTower(15, 32, [64, 32], use_content_embedding=False),
                         temperature=0.1).to(dev)


def test_forward_keys_loss_and_embeddings(dev):
    m = _small_model(dev)
    uf = {"numerical": torch.randn(8, 10, device=dev), "categorical": {}}
    itf = {"numerical": torch.randn(8, 15, device=dev), "categorical": {}}
    out = m(uf, itf)
    assert out["user_embedding"].shape == (8, 32) and out["item_embedding"].shape == (8, 32)
    assert out["similarity"].shape == (8,)
    out = m(uf, itf, compute_loss=True)
    assert out["loss"].ndim == 0 and out["loss"].item() >= 0
    e = m.get_user_embeddings({"numerical": torch.randn(4, 10, device=dev), "categorical": {}})
    assert torch.allclose(e.norm(dim=1), torch.ones(4, device=dev), atol=1e-5)
    neg = {"numerical": torch.randn(8 * 4, 15, device=dev), "categorical": {}}
    out = m(uf, itf, compute_loss=True, negative_items=neg)
    assert out["loss"].item() > 0


def test_save_load_roundtrip_and_eval_determinism(dev):
    UserTower, ItemTower, TwoTowerModel, _ = _mods()
    m = _small_model(dev)
    m.eval()
    with tempfile.TemporaryDirectory() as td:
        path = Path(td) / "model.pth"
        torch.manual_seed(42)
        x = {"numerical": torch.randn(4, 10).to(dev), "categorical": {}}
        a = m.get_user_embeddings(x)
        m.save_model(str(path))
        m2 = TwoTowerModel(UserTower(10, 32, [64, 32]), ItemTower(15, 32, [64, 32], use_content_embedding=False),
                           temperature=0.1)
        m2.load_model(str(path))
        m2.to(dev).eval()
        b = m2.get_user_embeddings(x)
        assert torch.allclose(a, b, atol=1e-4)
        assert torch.equal(m.get_user_embeddings(x), a)


def test_factory(dev):
    _, _, TwoTowerModel, create = _mods()
    m = create({"embedding_dim": 64, "temperature": 0.05})
    assert isinstance(m, TwoTowerModel) and m.temperature == 0.05
    assert isinstance(create({}), TwoTowerModel)


def test_embedding_quality_after_training(dev):
    """tests/test_two_tower_model.py:312-361 with torch.optim.Adam on the fused model."""
    UserTower, ItemTower, TwoTowerModel, _ = _mods()
    torch.manual_seed(0)
    m = TwoTowerModel(UserTower(10, 32, [32]), ItemTower(10, 32, [32], use_content_embedding=False),
                      temperature=0.1).to(dev)
    opt = torch.optim.Adam(m.parameters(), lr=0.01)
    for _ in range(10):
        out = m({"numerical": torch.randn(16, 10, device=dev), "categorical": {}},
                {"numerical": torch.randn(16, 10, device=dev), "categorical": {}}, compute_loss=True)
        opt.zero_grad()
        out["loss"].backward()
        opt.step()
    m.eval()
    base = torch.randn(1, 10, device=dev)
    e1 = m.get_user_embeddings({"numerical": base, "categorical": {}})
    e2 = m.get_user_embeddings({"numerical": base + 0.01 * torch.randn(1, 10, device=dev), "categorical": {}})
    assert torch.sum(e1 * e2) > 0.9
    emb = m.get_user_embeddings({"numerical": torch.randn(100, 10, device=dev), "categorical": {}})
    assert torch.var(emb) > 0.01


def test_dropout_train_mode_statistics(dev):
    UserTower, _, _, _ = _mods()
    t = UserTower(10, 256, [256, 256], dropout_rate=0.5).to(dev)
    x = torch.randn(512, 10, device=dev)
    a, b = t(x), t(x)
    assert not torch.allclose(a, b)  # fresh masks per call
    t.eval()
    assert torch.equal(t(x), t(x))


def test_cpu_tensors_raise():
    UserTower, _, _, _ = _mods()
    t = UserTower(10, 32, [64, 32])
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        t(torch.randn(4, 10))


def test_tower_forward_is_fp32_class(dev):
    """The tower kernels take fp32 products on the bf16 MFMA (three-piece split,
    DESIGN.md §5 note i). Against a float64 evaluation of the same module
    (k = 256 and 128 reductions, eval BatchNorm, ReLU, final L2 normalise), the
    device output's max error must stay within 4x the max error of torch's own
    fp32 CPU forward and below 2e-6 absolute: fp32-class, not bit-compatible —
    the split drops three piece products of order <= 2^-23 and the MFMA's
    blocked summation order differs from torch's."""
    import copy
    UserTower, _, _, _ = _mods()
    torch.manual_seed(7)
    t = UserTower(256, 128, [256, 128], dropout_rate=0.0)
    for mod in t.mlp:
        if isinstance(mod, nn.BatchNorm1d):
            mod.running_mean.uniform_(-0.5, 0.5)
            mod.running_var.uniform_(0.5, 2.0)
    t.eval()
    x = torch.randn(4096, 256)
    ref_mlp = copy.deepcopy(t.mlp).double()
    with torch.no_grad():
        z64 = ref_mlp(x.double())
        ref = z64 / z64.norm(dim=1, keepdim=True)
        z32 = copy.deepcopy(t.mlp)(x)
        cpu32 = z32 / z32.norm(dim=1, keepdim=True)
        got = t.to(dev)(x.to(dev)).cpu().double()
    err_dev = (got - ref).abs().max().item()
    err_cpu = (cpu32.double() - ref).abs().max().item()
    assert err_dev <= 4 * err_cpu + 1e-7, (err_dev, err_cpu)
    assert err_dev < 2e-6, err_dev
