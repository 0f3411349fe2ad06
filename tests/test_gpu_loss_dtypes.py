"""Fused loss on 16-bit embeddings (config C5 is bf16, D=256): inputs are
widened to fp32 on load, so the result must equal the fp32 reference math run
on the same (rounded) values — loss within 1e-4 relative (north star), grads to
fp32 accumulation-order noise; also B not a multiple of the 256-row span."""
import numpy as np
import pytest
import torch

from oracle import two_tower as orc
from rtrec_amd import kernels

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("b,d,n_neg", [(512, 256, 0), (300, 128, 16), (1024, 64, 4)])
def test_mixed_loss_dtypes(device, dtype, b, d, n_neg):
    g = torch.Generator().manual_seed(b + d + n_neg)
    u = torch.nn.functional.normalize(torch.randn(b, d, generator=g), dim=1).to(dtype)
    p = torch.nn.functional.normalize(torch.randn(b, d, generator=g), dim=1).to(dtype)
    q = torch.nn.functional.normalize(torch.randn(b * n_neg, d, generator=g), dim=1).to(dtype) if n_neg else None
    tau = 0.05
    ub, ib = torch.tensor([0.1]), torch.tensor([-0.05])
    # reference on the rounded values in fp32 (reference math, torch autograd)
    uu = u.float().requires_grad_()
    pp = p.float().requires_grad_()
    qq = q.float().requires_grad_() if q is not None else None
    ib_loss = orc.in_batch_negative_loss(uu, pp, tau)
    if q is not None:
        ex = orc.contrastive_loss(uu, pp, qq, tau, ub, ib)
        total = 0.7 * ex + 0.3 * ib_loss
    else:
        total = ib_loss
    total.backward()
    loss, du, dp, dq, _, _ = kernels.twotower_loss(u.to(device), p.to(device), q.to(device) if q is not None else None,
                                                   tau, ub.to(device), ib.to(device))
    torch.cuda.synchronize()
    np.testing.assert_allclose(loss[0].item(), total.item(), rtol=1e-4)
    np.testing.assert_allclose(loss[2].item(), ib_loss.item(), rtol=1e-4)
    sc = float(uu.grad.abs().max())
    np.testing.assert_allclose(du.cpu().numpy(), uu.grad.numpy(), rtol=0, atol=1e-4 * sc)
    np.testing.assert_allclose(dp.cpu().numpy(), pp.grad.numpy(), rtol=0, atol=1e-4 * float(pp.grad.abs().max()))
    if q is not None:
        np.testing.assert_allclose(dq.cpu().numpy(), qq.grad.numpy(), rtol=0,
                                   atol=1e-4 * float(qq.grad.abs().max()))


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("world,b,d", [(4, 256, 256), (3, 96, 128)])
def test_rect_inbatch_loss_equals_sharded_square(device, dtype, world, b, d):
    """rt_inbatch_loss_fwd_bwd on each simulated rank (b local users vs all
    world·b items, label offset r·b) averages to the square reference loss."""
    g = torch.Generator().manual_seed(world * b + d)
    U = torch.nn.functional.normalize(torch.randn(world * b, d, generator=g), dim=1).to(dtype)
    P = torch.nn.functional.normalize(torch.randn(world * b, d, generator=g), dim=1).to(dtype)
    uu, pp = U.float().requires_grad_(), P.float().requires_grad_()
    ref = orc.in_batch_negative_loss(uu, pp, 0.05)
    ref.backward()
    Ud, Pd = U.to(device), P.to(device)
    tot, dps = 0.0, torch.zeros(world * b, d, device=device)
    for r in range(world):
        loss, du, dp = kernels.inbatch_loss(Ud[r * b:(r + 1) * b], Pd, 0.05, label_offset=r * b)
        tot += loss[0].item() / world
        dps += dp / world
        np.testing.assert_allclose((du / world).cpu().numpy(), uu.grad[r * b:(r + 1) * b].numpy(), rtol=0,
                                   atol=1e-4 * float(uu.grad.abs().max()))
    np.testing.assert_allclose(tot, ref.item(), rtol=1e-4)
    np.testing.assert_allclose(dps.cpu().numpy(), pp.grad.numpy(), rtol=0, atol=1e-4 * float(pp.grad.abs().max()))
