"""Split-weight planes (DESIGN.md §5 note i, round 6): each weight's three
bf16 pieces are written once per chain by a side task of the launch before the
one that uses them, instead of being split in registers by every block of the
forward and dz launches. The pieces are the bits split3 gives, so the tower
forward must be bit-identical with the planes on and off, and the C2 train
step equal up to the fp32 atomics of its last dW launch."""
import copy

import pytest
import torch

from rtrec_amd.models import fused

pytestmark = pytest.mark.gpu


def _model(device, dropout=0.2):
    from rtrec_amd.training.utils import create_two_tower_model_for_training
    torch.manual_seed(3)
    cfg = {"embedding_dim": 128, "hidden_layers": [256, 128], "dropout_rate": dropout, "temperature": 0.05}
    return create_two_tower_model_for_training(3, 20, cfg).to(device)


@pytest.fixture
def planes_switch():
    keep = (fused.SPLIT_W_PLANES, fused.SPLIT_W_PLANES_FWD, fused.SPLIT_W_PLANES_DZ)
    fused.SPLIT_W_PLANES_FWD = fused.SPLIT_W_PLANES_DZ = True
    yield
    fused.SPLIT_W_PLANES, fused.SPLIT_W_PLANES_FWD, fused.SPLIT_W_PLANES_DZ = keep


def test_tower_forward_bit_identical_with_planes(device, planes_switch):
    """Eval and train-mode tower forwards (k = 256 / 128 layers read the
    planes) equal the in-register split bit for bit."""
    m = _model(device)
    g = torch.Generator(device=device).manual_seed(1)
    items = torch.randn(4096, 20, device=device, generator=g)
    users = torch.randn(1000, 3, device=device, generator=g)
    outs = {}
    for on in (False, True):
        fused.SPLIT_W_PLANES = on
        m.eval()
        with torch.no_grad():
            e = (m.item_tower(items), m.user_tower(users))
        outs[on] = e
    for a, b in zip(outs[False], outs[True]):
        assert torch.equal(a, b)


def test_train_step_with_planes_matches_register_split(device, planes_switch):
    """The C2-shaped fused step's gradients (B 1024, 16 negatives, emb 128,
    dropout 0.2) with the planes on and off: the loss within 1e-12 relative
    (its fp64 atomics may reorder), every parameter gradient within 1e-5 of
    its tensor's max (the last dW launch adds its tiles with fp32 atomics)."""
    from rtrec_amd.training.fused_step import FusedTrainStep
    m0 = _model(device)
    g = torch.Generator(device=device).manual_seed(2)
    ut = torch.randn(6040, 3, device=device, generator=g)
    mt = torch.randn(3416, 20, device=device, generator=g)
    u = torch.randint(0, 6040, (1024,), device=device, generator=g)
    pn = torch.randint(0, 3416, (1024 * 17,), device=device, generator=g)
    p, n = pn[:1024], pn[1024:].view(1024, 16)
    res = {}
    for on in (False, True):
        fused.SPLIT_W_PLANES = on
        m = copy.deepcopy(m0)
        st = FusedTrainStep(m, dropout_seed=77)
        m.train()
        st._ensure_clean()
        st._grads(ut, mt, mt, u, p, n)
        torch.cuda.synchronize()
        res[on] = (float(st.loss_buf[0].item()), [st.slab.grad[o:e].clone() for o, e in st.slab.bounds])
    la, lb = res[False][0], res[True][0]
    assert abs(la - lb) <= 1e-12 * abs(la), (la, lb)
    for ga, gb in zip(res[False][1], res[True][1]):
        tol = 1e-5 * float(ga.abs().max()) + 1e-30
        assert float((ga - gb).abs().max()) <= tol
