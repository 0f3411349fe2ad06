"""Config C5 at the bench's own scale: a 12.5M-row x 256 bf16
shard — 6.4 GB, row byte offsets past 4 GiB — gathered by the product kernel
(rt_gather_rows, csrc/gather.hip: 64-bit row offsets) with 16.8M ids and
compared bit for bit with torch indexing; and the C5 in-batch step
(sharded_inbatch_step) on that full shard against the reference loss math
(src/models/two_tower.py:453-479) in fp32 on the gathered rows."""
import numpy as np
import pytest
import torch

from rtrec_amd import kernels
from rtrec_amd.dist.sharded import sharded_inbatch_step

pytestmark = pytest.mark.gpu

ROWS, DIM = 12_500_000, 256


@pytest.fixture(scope="module")
def shard(device):
    g = torch.Generator(device=device).manual_seed(2000)
    t = torch.empty((ROWS, DIM), dtype=torch.bfloat16, device=device)
    step = 1_000_000
    for r0 in range(0, ROWS, step):  # bounded fp32 temporaries
        t[r0:r0 + step] = (torch.randn(min(step, ROWS - r0), DIM, device=device, generator=g) * 0.01)
    t[-1] = 7.0                      # the last row (byte offset 6.4e9) is recognisable
    yield t
    del t
    torch.cuda.empty_cache()


def test_c5_gather_full_shard_bit_exact(device, shard):
    """16.8M uniform ids over the whole 12.5M-row shard (two thirds of them
    beyond the 4 GiB byte offset), plus the last row and row 0 planted: the
    gathered rows equal ``shard[ids]`` bit for bit."""
    g = torch.Generator(device=device).manual_seed(3000)
    n_ids = 16_777_216
    ids = torch.randint(0, ROWS, (n_ids,), device=device, generator=g)
    ids[:4] = torch.tensor([ROWS - 1, 0, ROWS - 1, 8_388_608], device=device)  # 8,388,608 x 512 B = 4 GiB
    out = kernels.gather_rows(shard, ids)
    torch.cuda.synchronize()
    assert out.shape == (n_ids, DIM) and out.dtype == torch.bfloat16
    assert bool((out[0].float() == 7.0).all())
    chunk = 2_097_152
    for c0 in range(0, n_ids, chunk):
        sl = slice(c0, c0 + chunk)
        assert torch.equal(out[sl].view(torch.int16), shard[ids[sl]].view(torch.int16)), c0
    del out
    torch.cuda.empty_cache()


def test_c5_gather_shard_window_of_global_ids(device, shard):
    """The same shard as rank 3 of 8 (global rows [37.5M, 50M)): global ids over
    the 100M-row table give the shard's rows inside the window and zero rows
    outside it (counted as out of range), bit for bit."""
    g = torch.Generator(device=device).manual_seed(3001)
    n_ids, begin = 4_194_304, 3 * ROWS
    ids = torch.randint(0, 8 * ROWS, (n_ids,), device=device, generator=g)
    ids[:2] = torch.tensor([begin + ROWS - 1, begin], device=device)
    oob = torch.zeros(1, dtype=torch.int32, device=device)
    out = kernels.gather_rows(shard, ids, row_begin=begin, oob=oob)
    loc = ids - begin
    inside = (loc >= 0) & (loc < ROWS)
    ref = torch.zeros_like(out)
    ref[inside] = shard[loc[inside]]
    torch.cuda.synchronize()
    assert torch.equal(out.view(torch.int16), ref.view(torch.int16))
    assert int(oob.item()) == int((~inside).sum().item())


def test_c5_sharded_step_full_shard_matches_fp32_reference(device, shard):
    """sharded_inbatch_step on the full 12.5M-row shard (B = 8192 users, D = 256,
    bf16, tau 0.05; N = 1 runs the same exchange code without collectives):
    loss within 1e-4 relative of the fp32 reference on the gathered rows,
    gradients within 1e-4 of their max magnitude."""
    g = torch.Generator(device=device).manual_seed(3002)
    b, tau = 8192, 0.05
    ids = torch.randint(0, ROWS, (b,), device=device, generator=g)
    ids[0] = ROWS - 1
    u = torch.nn.functional.normalize(torch.randn(b, DIM, device=device, generator=g), dim=1).to(torch.bfloat16)
    loss, du, dp = sharded_inbatch_step(shard, 0, u, ids, tau)
    rows = shard[ids]
    torch.cuda.synchronize()
    uu = u.float().cpu().requires_grad_()
    pp = rows.float().cpu().requires_grad_()
    ref = torch.nn.functional.cross_entropy(uu @ pp.t() / tau, torch.arange(b))
    ref.backward()
    np.testing.assert_allclose(float(loss[0].item()), float(ref), rtol=1e-4)
    rdu, rdp = uu.grad.numpy(), pp.grad.numpy()
    np.testing.assert_allclose(du.float().cpu().numpy(), rdu, rtol=0, atol=1e-4 * np.abs(rdu).max())
    np.testing.assert_allclose(dp.float().cpu().numpy(), rdp, rtol=0, atol=1e-4 * np.abs(rdp).max())
