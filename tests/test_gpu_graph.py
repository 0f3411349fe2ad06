"""hipGraph capture/replay of the fused C2 step (what bench.py times): with
dropout off, replaying the captured step over fresh ids in the static buffers
gives the same losses and parameters as the eager step (to the run-to-run
noise of the fp32/fp64 atomics that accumulate dW and the BN column sums).
``capture`` restores the training state its warmup steps touched (default), or
keeps them (``restore=False``)."""
import copy

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(device):
    from rtrec_amd.data.movielens import build_batches, feature_tables, synthetic_movielens
    from rtrec_amd.training.utils import create_two_tower_model_for_training
    data = synthetic_movielens(n_users=500, n_movies=600, n_ratings=30000, seed=4)
    uf, mf = feature_tables(data)
    bu, bp, bn = build_batches(data.train_interactions, data.num_movies, 256, 8, 4, seed=9)
    ut, mt = torch.from_numpy(uf).to(device), torch.from_numpy(mf).to(device)
    batches = [tuple(torch.from_numpy(x[i]).to(device) for x in (bu, bp, bn)) for i in range(4)]
    torch.manual_seed(0)
    m1 = create_two_tower_model_for_training(3, 20, {"embedding_dim": 64, "hidden_layers": [128, 64],
                                                     "dropout_rate": 0.0, "temperature": 0.05}).to(device)
    return ut, mt, batches, m1


def _check(m1, m2, ref, got):
    torch.cuda.synchronize()
    for a, c in zip(ref, got):
        torch.testing.assert_close(c, a, rtol=1e-6, atol=1e-7)
    for a, c in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(c, a, rtol=1e-5, atol=1e-6)
    for a, c in zip(m1.buffers(), m2.buffers()):
        torch.testing.assert_close(c, a, rtol=1e-5, atol=1e-6)


def test_graph_replay_matches_eager(device):
    from rtrec_amd.training.fused_step import FusedTrainStep
    ut, mt, batches, m1 = _setup(device)
    m2 = copy.deepcopy(m1)
    eager = FusedTrainStep(m1)
    ref = [eager(ut, mt, mt, user_ids=b[0], pos_ids=b[1], neg_ids=b[2]).clone() for b in batches]
    g = FusedTrainStep(m2)
    st = tuple(t.clone() for t in batches[1])
    g.capture(ut, mt, mt, user_ids=st[0], pos_ids=st[1], neg_ids=st[2], warmup=2)  # state restored
    got = []
    for b in batches:
        for dst, src in zip(st, b):
            dst.copy_(src)
        got.append(g.replay().clone())
    _check(m1, m2, ref, got)


def test_graph_capture_keeps_warmup_when_asked(device):
    from rtrec_amd.training.fused_step import FusedTrainStep
    ut, mt, batches, m1 = _setup(device)
    m2 = copy.deepcopy(m1)
    eager = FusedTrainStep(m1)
    ref = []
    for b in [batches[0], batches[0], batches[1], batches[2], batches[3]]:
        ref.append(eager(ut, mt, mt, user_ids=b[0], pos_ids=b[1], neg_ids=b[2]).clone())
    g = FusedTrainStep(m2)
    st = tuple(t.clone() for t in batches[0])
    g.capture(ut, mt, mt, user_ids=st[0], pos_ids=st[1], neg_ids=st[2], warmup=2, restore=False)
    got = []
    for b in batches[1:]:
        for dst, src in zip(st, b):
            dst.copy_(src)
        got.append(g.replay().clone())
    _check(m1, m2, ref[2:], got)


@pytest.mark.parametrize("backend", ["gloo", "nccl"])
def test_two_graph_data_parallel_capture(device, backend):
    """The data-parallel form bench.py replays at N > 1: with a process group the
    step is captured as two graphs (gradients; clip+Adam) with the all-reduce
    of the flat grad slab launched eagerly between them. Exercised here with a
    one-rank group (the all-reduce is then the identity): gloo (SUM + scale)
    and nccl = RCCL (ReduceOp.AVG, the path of the multi-GPU bench); the
    replays equal the eager single-process steps."""
    import socket

    import torch.distributed as dist

    from rtrec_amd.training.fused_step import FusedTrainStep
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    kw = {"device_id": torch.device(device)} if backend == "nccl" else {}
    dist.init_process_group(backend, init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, **kw)
    try:
        ut, mt, batches, m1 = _setup(device)
        m2 = copy.deepcopy(m1)
        eager = FusedTrainStep(m1)
        ref = [eager(ut, mt, mt, user_ids=b[0], pos_ids=b[1], neg_ids=b[2]).clone() for b in batches]
        g = FusedTrainStep(m2, process_group=dist.group.WORLD)
        st = tuple(t.clone() for t in batches[0])
        g.capture(ut, mt, mt, user_ids=st[0], pos_ids=st[1], neg_ids=st[2], warmup=1)
        assert g.graph_update is not None
        got = []
        for b in batches:
            for dst, src in zip(st, b):
                dst.copy_(src)
            got.append(g.replay().clone())
        _check(m1, m2, ref, got)
    finally:
        dist.destroy_process_group()


def test_step_after_autograd_backward_matches_fresh_step(device):
    """an autograd backward through the same model between fused
    steps accumulates into the shared grad slab. The next fused step must see a
    clean slab (it re-zeroes when slab.grad_gen moved), so it equals the same
    step on an untouched copy of the model."""
    from rtrec_amd.training.fused_step import FusedTrainStep
    ut, mt, batches, m1 = _setup(device)
    m2 = copy.deepcopy(m1)
    s1, s2 = FusedTrainStep(m1), FusedTrainStep(m2)
    b = batches[0]
    s1(ut, mt, mt, user_ids=b[0], pos_ids=b[1], neg_ids=b[2])
    s2(ut, mt, mt, user_ids=b[0], pos_ids=b[1], neg_ids=b[2])
    # autograd through the HIP towers of m1 only: grads land in m1's slab
    m1.train()
    u = m1.user_tower(ut[:64].contiguous())
    p = m1.item_tower(mt[:64].contiguous())
    m1.in_batch_negative_loss(u, p).backward()
    assert float(s1.slab.grad.abs().sum()) > 0.0
    # BN running stats moved in m1's towers: copy them over so only the slab differs
    with torch.no_grad():
        for a, c in zip(m2.buffers(), m1.buffers()):
            a.copy_(c)
    b = batches[1]
    ref = s2(ut, mt, mt, user_ids=b[0], pos_ids=b[1], neg_ids=b[2]).clone()
    got = s1(ut, mt, mt, user_ids=b[0], pos_ids=b[1], neg_ids=b[2]).clone()
    _check(m2, m1, [ref], [got])


def _feeder_pair(device, dropout):
    from rtrec_amd.data.movielens import synthetic_movielens
    from rtrec_amd.training.datasets.movielens import DeviceFeeder
    from rtrec_amd.training.fused_step import FusedTrainStep
    from rtrec_amd.training.utils import create_two_tower_model_for_training
    data = synthetic_movielens(seed=0)
    torch.manual_seed(7)
    cfg = {"embedding_dim": 64, "hidden_layers": [256, 128], "dropout_rate": dropout, "temperature": 0.05}
    m1 = create_two_tower_model_for_training(3, 20, cfg)
    m2 = copy.deepcopy(m1)
    m1.to(device)
    m2.to(device)
    mk = lambda: DeviceFeeder(data.train_interactions, data.users, data.movies, num_negatives=16,  # noqa: E731
                              batch_size=256, device=device, seed=5)
    # the same dropout seed base: masks then depend only on the device step counter
    return (m1, m2, mk(), mk(), FusedTrainStep(m1, dropout_seed=1234), FusedTrainStep(m2, dropout_seed=1234))


def test_feeder_graph_epoch_matches_eager(device):
    """FeederGraph (batch rows at a device cursor, on-device negatives and the
    fused step as one hipGraph per batch) reproduces the eager feeder-driven
    loop WITH dropout 0.2: the same batches (ids compared
    exactly) and the same per-batch losses. Eager and captured steps draw
    their masks from the same per-chain seed bases plus the device step
    counter, so step t masks agree whichever way the step runs."""
    from rtrec_amd.training.fused_step import FeederGraph
    m1, m2, fa, fb, sa, sb = _feeder_pair(device, 0.2)
    nb = 40
    eager, last = [], None
    for i, b in enumerate(fa):
        if i == nb:
            break
        eager.append(float(sa(b["user_table"], b["item_table"], b["item_table"], user_ids=b["user_ids"],
                              pos_ids=b["pos_ids"], neg_ids=b["neg_ids"])[0].item()))
        last = b
    fg = FeederGraph(sb, fb)
    got = fg.run_epoch(max_batches=nb).cpu().numpy()
    assert fb.epoch == 1
    assert torch.equal(fg.users, last["user_ids"]) and torch.equal(fg.pos, last["pos_ids"])
    assert torch.equal(fg.neg, last["neg_ids"])
    # The last dW launch of a step adds its tiles with fp32 atomics, so two runs
    # of the SAME eager loop already differ in the last bits of some gradients,
    # and Adam's normalised update plus dropout amplify that over the epoch:
    # measured on the GPU (profiles/r06_dropout_determinism.txt, 40 steps at
    # p = 0.2) eager vs eager 4.6e-5 loss relative / 2.1e-3 max weight, eager vs
    # graph 2.3e-5 / 6.0e-4 (p = 0: 5e-8 / 2e-6). A mask mismatch moves the
    # loss by ~1e-2 at the first step. Bars: the first 5 steps within 1e-5
    # relative, every step within 2e-4, weights within 5e-3 (vs ~1.4 moved).
    eager = np.asarray(eager)
    np.testing.assert_allclose(got[:5], eager[:5], rtol=1e-5)
    np.testing.assert_allclose(got, eager, rtol=2e-4)
    for (k, v1), v2 in zip(m1.state_dict().items(), m2.state_dict().values()):
        diff = float((v1.float() - v2.float()).abs().max()) if v1.numel() else 0.0
        assert diff <= 5e-3, (k, diff)


def test_dropout_masks_change_per_step_with_fixed_seed_base(device):
    """A fixed seed base does not freeze the masks: consecutive steps on the
    same batch with dropout on give different losses, and two step objects with
    different seed bases differ at the same step."""
    from rtrec_amd.training.fused_step import FusedTrainStep
    m1, m2, fa, _, sa, _ = _feeder_pair(device, 0.2)
    b = next(iter(fa))
    args = (b["user_table"], b["item_table"], b["item_table"])
    kw = dict(user_ids=b["user_ids"], pos_ids=b["pos_ids"], neg_ids=b["neg_ids"])
    m3 = copy.deepcopy(m2)
    s3 = FusedTrainStep(m3, dropout_seed=99)
    l1 = float(sa(*args, **kw)[0].item())
    l3 = float(s3(*args, **kw)[0].item())
    # other masks move the first-step loss far beyond the 1e-5 bar of the graph test
    assert abs(l1 - l3) > 1e-4 * abs(l1), (l1, l3)
    s0 = FusedTrainStep(copy.deepcopy(m2), dropout_seed=1234, lr=0.0)
    la, lb = float(s0(*args, **kw)[0].item()), float(s0(*args, **kw)[0].item())
    assert la != lb  # lr 0: the weights stay, only the step counter (and so the masks) moved


def test_feeder_graph_survives_larger_validation_batch(device):
    """a validation batch larger than the training batch
    between two FeederGraph epochs grows the shared loss workspace of the
    autograd path; the captured step owns its workspace, so the second epoch
    still equals a twin run with no validation in between."""
    from rtrec_amd.training.fused_step import FeederGraph
    m1, m2, fa, fb, sa, sb = _feeder_pair(device, 0.0)
    g1, g2 = FeederGraph(sa, fa), FeederGraph(sb, fb)
    g1.run_epoch(max_batches=6)
    g2.run_epoch(max_batches=6)
    with torch.no_grad():  # the reference validate(): in-batch loss, eval mode, a 4x larger batch
        m1.eval()
        ut, mt = fa.user_table, fa.item_table
        gen = torch.Generator(device=device).manual_seed(3)
        u = m1.user_tower(ut[torch.randint(0, ut.shape[0], (1024,), device=device, generator=gen)])
        p = m1.item_tower(mt[torch.randint(0, mt.shape[0], (1024,), device=device, generator=gen)])
        float(m1.in_batch_negative_loss(u, p))
        junk = [torch.full((1 << 20,), float("nan"), device=device) for _ in range(8)]  # reuse freed blocks
        m1.train()
    got = g1.run_epoch(max_batches=6).cpu().numpy()
    want = g2.run_epoch(max_batches=6).cpu().numpy()
    del junk
    assert np.isfinite(got).all()
    np.testing.assert_allclose(got, want, rtol=1e-5)
