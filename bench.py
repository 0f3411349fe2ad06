#!/usr/bin/env python3
"""Benchmark: user-item pairs scored/sec (train) + top-K queries/sec, emb_dim=128.

Headline (BASELINE.json configs[1], "C2"): the MovieLens-1M two-tower training
step at emb_dim=128, batch 1024, 16 explicit negatives per user, hidden
[256,128], dropout 0.2, tau 0.05, Adam(1e-3, wd 1e-5), clip 1.0
(scripts/train_movielens.py:39-122 → TwoTowerTrainer.train_epoch,
src/training/trainers/two_tower.py:98-146) on an ML-1M-shaped synthetic
stream (ratings.dat is not available). One step = feature-row gather (fused)
+ user/pos/neg tower forward + fused 0.7·contrastive + 0.3·in-batch loss
forward/backward + tower backward + clip + Adam, all on the MI355X kernels.
pairs/step = B² (in-batch) + B·N (explicit) per GPU; N GPUs run data-parallel
replicas on their own batches with one RCCL all-reduce of the flat grad slab
(weak scaling).

Extras on the same line (rank 0): Flat-IP top-K QPS at config 3 (6,040 users x
3,416 items, fp32, k=10) and a config-4 shard (65,536 queries x 125,000
items, fp16, k=100), the HBM row-gather rate (config-5 table shard, bf16
rows of 256), the config-5 in-batch scoring CE (8,192 x 8,192 x 256 bf16,
forward and forward+backward on the 16-bit MFMA), the live roofline of the
dominant kernel, and the CPU baseline (the oracle's torch-CPU restatement of
the same step on this host's cores).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       torchrun --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "real-time-recommendation-system-with-feature-store_amd")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

PEAK_F32_TFLOPS = 157.3   # MI355X dense fp32 (MFMA = vector rate), MI355X_MICROARCH.md
PEAK_BF16_TFLOPS = 2500.0  # dense bf16/fp16 MFMA
PEAK_HBM_GBS = 8000.0      # HBM3E spec


SPACER_CYCLES = 200_000  # ≈0.1 ms GPU spin ahead of each timed launch (profiling.KernelTimer)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def dist_setup(n_gpus):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        # rehearsal knobs for a one-GPU box (never set by the driver): every rank
        # on cuda:0 (RCCL refuses two ranks on one device, so collectives then
        # go through gloo)
        if os.environ.get("RTREC_BENCH_SAME_GPU") == "1":
            local = 0
        backend = os.environ.get("RTREC_BENCH_BACKEND", "nccl")
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
        return dist, rank, world, torch.device("cuda", local)
    return None, 0, 1, torch.device("cuda", 0)


def _batch(dev, u, p, n):
    """Device ids of one batch; positive and negative item ids share one buffer
    (negatives right after positives: the item tower reads them as one id list)."""
    pn = torch.from_numpy(np.concatenate([p.reshape(-1), n.reshape(-1)])).to(dev)
    return torch.from_numpy(u).to(dev), pn[:p.size].view(p.shape), pn[p.size:].view(n.shape)


def c2_setup(dev, rank, n_batches, dropout=0.2):
    """The C2 workload: ML-1M-shaped tables resident on the device, id batches
    (B=1024, N=16), the training-factory model (emb 128, hidden [256,128]).
    tests/test_gpu_c2_fullsize.py runs this same setup at dropout 0 against
    the oracle."""
    from rtrec_amd.data.movielens import build_batches, feature_tables, synthetic_movielens
    from rtrec_amd.training.utils import create_two_tower_model_for_training
    data = synthetic_movielens(seed=0)
    uf, mf = feature_tables(data)
    bu, bp, bn = build_batches(data.train_interactions, data.num_movies, 1024, 16, n_batches, seed=100 + rank)
    torch.manual_seed(1234)
    model = create_two_tower_model_for_training(3, 20, {"embedding_dim": 128, "hidden_layers": [256, 128],
                                                        "dropout_rate": dropout, "temperature": 0.05})
    tables = (torch.from_numpy(uf).to(dev), torch.from_numpy(mf).to(dev))
    batches = [_batch(dev, bu[i], bp[i], bn[i]) for i in range(n_batches)]
    return model, tables, batches, (uf, mf, bu, bp, bn)


def _host_cores() -> int:
    return len(os.sched_getaffinity(0))


def _cgroup_cpu_quota():
    """CPUs granted by this process's cgroup CPU quota (cgroup v2 cpu.max or v1
    cfs_quota_us / cfs_period_us), None when unlimited or unreadable."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            return max(1, -(-int(q) // int(per)))
        return None
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        return max(1, -(-q // per)) if q > 0 else None
    except (OSError, ValueError):
        return None


def _cpu_cores() -> int:
    """The cores this process can actually run on: the affinity set, capped by
    the cgroup CPU quota. On the GPU box the affinity set is the whole 256-core
    host but the quota is 16 CPUs; torch.set_num_threads(256) there ran one C2
    step in 30.7 s (profiles/r03s1_bench.json), 16x oversubscribed, against
    ~90 ms on the 16 granted cores."""
    q = _cgroup_cpu_quota()
    if q is None and os.environ.get("OMP_NUM_THREADS", "").isdigit():
        q = int(os.environ["OMP_NUM_THREADS"]) or None  # the box's documented per-job CPU share
    n = _host_cores()
    return min(n, q) if q else n


# The reference's own C2 step on its CPU path, measured in the survey container
# ("Full mixed-loss train step, B=1024, N=16, emb 128, hidden
# [256,128]: 106 ms", src/training/trainers/two_tower.py:98-146). The only
# number BASELINE.md holds for this exact metric and config (the reference
# publishes none for it): vs_baseline = value / this.
BASELINE_MD_C2_MS = 106.0
BASELINE_MD_C2_PAIRS_PER_S = (1024 * 1024 + 1024 * 16) / (BASELINE_MD_C2_MS * 1e-3)


def cpu_baseline(host, budget_s=10.0, threads=None):
    """The oracle's torch-CPU restatement of the reference step (same math as
    src/training/trainers/two_tower.py:98-146) on a bounded sample of C2 batches,
    on every core this process may run on (torch.set_num_threads(
    len(os.sched_getaffinity(0))), capped by the cgroup CPU quota: _cpu_cores)."""
    from oracle import two_tower as orc
    from rtrec_amd.training.utils import create_two_tower_model_for_training
    uf, mf, bu, bp, bn = host
    threads = threads or _cpu_cores()
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    torch.manual_seed(1234)
    model = create_two_tower_model_for_training(3, 20, {"embedding_dim": 128, "hidden_layers": [256, 128],
                                                        "dropout_rate": 0.2, "temperature": 0.05})
    us = {k: v.clone() for k, v in model.user_tower.state_dict().items()}
    its = {k: v.clone() for k, v in model.item_tower.state_dict().items()}
    biases = {"user_bias": torch.zeros(1), "item_bias": torch.zeros(1)}
    opt = {}
    steps, t0 = 0, time.perf_counter()
    while True:
        i = steps % bu.shape[0]
        u = torch.from_numpy(uf[bu[i]])
        p = torch.from_numpy(mf[bp[i]])
        n = torch.from_numpy(mf[bn[i]]).view(1024, 16, 20)
        orc.train_step(us, its, biases, opt, u, p, n, temperature=0.05, dropout_p=0.2)
        steps += 1
        el = time.perf_counter() - t0
        if el >= budget_s or steps >= 200:
            break
    pairs = steps * (1024 * 1024 + 1024 * 16)
    torch.set_num_threads(prev)
    return {"value": pairs / el, "unit": "pairs/s", "cores": threads, "threads": threads,
            "host_cores": _host_cores(), "cgroup_cpu_quota": _cgroup_cpu_quota(), "kind": "port",
            "sample": f"{steps} C2 train steps (B=1024, N=16, emb 128) of oracle/two_tower.train_step on "
                      f"torch-CPU with {threads} threads, {el:.1f}s", "ms_per_step": 1000.0 * el / steps}


def _cpu_topk(q, x, k, qblock=4096, xblock=65536):
    """Faiss-1.7.4-style exact IP top-k on the CPU (IndexFlatIP.search for
    nq >= 20: blocked sgemm + per-row selection): blocked torch.mm + torch.topk,
    fp32 (Faiss is fp32-only)."""
    out_s, out_i = [], []
    for q0 in range(0, q.shape[0], qblock):
        qb = q[q0:q0 + qblock]
        bs = bi = None
        for x0 in range(0, x.shape[0], xblock):
            sc = qb @ x[x0:x0 + xblock].T
            ts, ti = torch.topk(sc, min(k, sc.shape[1]), dim=1)
            ti += x0
            if bs is None:
                bs, bi = ts, ti
            else:
                cs, ci = torch.cat([bs, ts], 1), torch.cat([bi, ti], 1)
                bs, j = torch.topk(cs, k, dim=1)
                bi = torch.gather(ci, 1, j)
        out_s.append(bs)
        out_i.append(bi)
    return torch.cat(out_s), torch.cat(out_i)


def cpu_topk_baseline(budget_s=8.0):
    """The top-K half of the metric on the host: C3 at full size (6,040 x 3,416
    x 128, k=10) and C4 on a query sample (2,048 of the queries against the full
    1M-item corpus, k=100, fp32), QPS extrapolated from the sample; every core
    this process may run on."""
    threads = _cpu_cores()
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(7)
    out = {}
    q = torch.nn.functional.normalize(torch.randn(6040, 128, generator=g), dim=1)
    x = torch.nn.functional.normalize(torch.randn(3416, 128, generator=g), dim=1)
    _cpu_topk(q, x, 10)
    reps, t0 = 0, time.perf_counter()
    while reps < 3 or (time.perf_counter() - t0 < budget_s / 4 and reps < 50):
        _cpu_topk(q, x, 10)
        reps += 1
    el = (time.perf_counter() - t0) / reps
    out["topk_c3"] = {"qps": 6040 / el, "ms": el * 1e3, "threads": threads, "host_cores": _host_cores(),
                      "kind": "port", "sample": f"full C3 (6040x3416x128 fp32, k=10), {reps} reps: blocked "
                                                "torch.mm + torch.topk (Faiss IndexFlatIP sgemm path)"}
    x = torch.nn.functional.normalize(torch.randn(1_000_000, 128, generator=g), dim=1)
    q = torch.nn.functional.normalize(torch.randn(2048, 128, generator=g), dim=1)
    _cpu_topk(q[:256], x, 100)
    t0 = time.perf_counter()
    _cpu_topk(q, x, 100)
    el = time.perf_counter() - t0
    out["topk_c4"] = {"qps": 2048 / el, "ms_per_2048_queries": el * 1e3, "threads": threads,
                      "host_cores": _host_cores(), "kind": "port",
                      "sample": "2,048 queries x 1M-item corpus x 128 fp32, k=100 (C4 corpus; QPS extrapolated "
                                "from the sample; Faiss is fp32-only, the GPU leg runs f16)"}
    del x, q
    torch.set_num_threads(prev)
    return out


def topk_extras(dev):
    from rtrec_amd import kernels
    from rtrec_amd.profiling import TIMER
    out = {}
    g = torch.Generator(device=dev).manual_seed(7)
    # config 3: 6040 x 3416 fp32, k=10
    q = torch.nn.functional.normalize(torch.randn(6040, 128, device=dev, generator=g), dim=1)
    x = torch.nn.functional.normalize(torch.randn(3416, 128, device=dev, generator=g), dim=1)
    for _ in range(3):
        kernels.flatip_topk(q, x, 10)
    torch.cuda.synchronize()
    # wall clock of back-to-back calls (QPS), then the kernel timer's pass
    # (its GPU spin ahead of each launch must not count in the QPS)
    reps = 20
    t0 = time.perf_counter()
    for _ in range(reps):
        kernels.flatip_topk(q, x, 10)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / reps
    TIMER.enable(["flatip_topk"])
    for _ in range(reps):
        kernels.flatip_topk(q, x, 10)
    s = TIMER.summary()["flatip_topk"]
    TIMER.disable()
    out["topk_c3"] = {"qps": 6040 / el, "ms": el * 1e3, "kernel_ms": s["avg_ms"],
                      "tflops": s["flops"] / s["count"] / (s["avg_ms"] * 1e-3) / 1e12, "dtype": "f32", "k": 10,
                      "shape": "6040x3416x128"}
    # config 4 shard: 65,536 queries x 125,000 items (1M / 8 GPUs), fp16, k=100
    q = torch.nn.functional.normalize(torch.randn(65536, 128, device=dev, generator=g), dim=1).half()
    x = torch.nn.functional.normalize(torch.randn(125000, 128, device=dev, generator=g), dim=1).half()
    kernels.flatip_topk(q, x, 100)
    torch.cuda.synchronize()
    # kernel-timer pass first (it also brings the clocks up), then the wall clock
    # of back-to-back calls for the QPS
    reps = 10
    TIMER.enable(["flatip_topk"])
    for _ in range(3):
        kernels.flatip_topk(q, x, 100)
    s = TIMER.summary()["flatip_topk"]
    TIMER.disable()
    t0 = time.perf_counter()
    for _ in range(reps):
        kernels.flatip_topk(q, x, 100)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / reps
    tf = s["flops"] / s["count"] / (s["avg_ms"] * 1e-3) / 1e12
    tb, tsrc = pmc_traffic("flatip_topk_c4")
    out["topk_c4_shard"] = {"qps": 65536 / el, "ms": el * 1e3, "kernel_ms": s["avg_ms"], "tflops": tf,
                            "mfma_frac": tf / PEAK_BF16_TFLOPS, "dtype": "f16", "k": 100,
                            "shape": "65536x125000x128", "compulsory_bytes": 2 * (65536 + 125000) * 128 + 65536 * 100 * 12,
                            "traffic_per_call": tb, "traffic_source": tsrc}
    del q, x
    # config 5 gather: bf16 rows of 256 from a 12.5M-row shard, 16M ids per launch
    rows = 12_500_000
    table = torch.empty((rows, 256), dtype=torch.bfloat16, device=dev)
    table.view(torch.int16).random_(-30000, 30000, generator=g)
    ids = torch.randint(0, rows, (16_777_216,), device=dev, generator=g)
    outb = torch.empty((ids.numel(), 256), dtype=torch.bfloat16, device=dev)
    kernels.gather_rows(table, ids, out=outb)
    torch.cuda.synchronize()
    TIMER.enable(["gather_rows"])
    for _ in range(5):
        kernels.gather_rows(table, ids, out=outb)
    s = TIMER.summary()["gather_rows"]
    TIMER.disable()
    gbs = s["bytes"] / s["count"] / (s["avg_ms"] * 1e-3) / 1e9
    tb, tsrc = pmc_traffic("gather_c5")
    out["gather_c5"] = {"GBps": gbs, "hbm_frac": gbs / PEAK_HBM_GBS, "ms": s["avg_ms"], "ids": ids.numel(),
                        "row_bytes": 512, "algorithmic_bytes": 2 * 512 * ids.numel() + 8 * ids.numel(),
                        "traffic": tb, "traffic_source": tsrc}
    del table, ids, outb
    torch.cuda.empty_cache()
    # config 5 in-batch scoring: S = U·Pᵀ/τ over B=8192 users x 8192 items, D=256
    # bf16, CE forward + backward on the 16-bit MFMA path (rt_inbatch_loss_fwd_bwd)
    u = (torch.randn(8192, 256, device=dev, generator=g) * 0.06).to(torch.bfloat16)
    p = (torch.randn(8192, 256, device=dev, generator=g) * 0.06).to(torch.bfloat16)
    for grad in (False, True):
        kernels.inbatch_loss(u, p, 0.05, grad=grad)
        torch.cuda.synchronize()
        TIMER.enable(["inbatch_loss"])
        for _ in range(10):
            kernels.inbatch_loss(u, p, 0.05, grad=grad)
        s = TIMER.summary()["inbatch_loss"]
        TIMER.disable()
        tf = s["flops"] / s["count"] / (s["avg_ms"] * 1e-3) / 1e12
        out["inbatch_c5_" + ("fwd_bwd" if grad else "fwd")] = {
            "ms": s["avg_ms"], "tflops": tf, "mfma_frac": tf / PEAK_BF16_TFLOPS, "dtype": "bf16",
            "shape": "8192x8192x256", "flops": "algorithmic: 2BND fwd, 6BND fwd+bwd"}
    del u, p
    torch.cuda.empty_cache()
    return out


def c2_with_feeder(dev, steps=30):
    """The C2 step with the batch source inside the timed region: DeviceFeeder
    (device shuffle + rt_sample_negatives over the train-interaction CSR, fused
    gather ids) feeding FusedTrainStep — the reference spends ≈345 ms per
    1024-sample batch in its DataLoader here. Timed as the
    trainer runs it: one whole epoch of FeederGraph replays (batch rows at a
    device cursor, negatives, step, loss slot: one hipGraph per batch;
    per-epoch permutation included), and, for comparison, ``steps`` eager
    feeder-iterated steps."""
    from rtrec_amd.data.movielens import synthetic_movielens
    from rtrec_amd.training.datasets.movielens import DeviceFeeder
    from rtrec_amd.training.fused_step import FeederGraph, FusedTrainStep
    from rtrec_amd.training.utils import create_two_tower_model_for_training
    data = synthetic_movielens(seed=0)
    feeder = DeviceFeeder(data.train_interactions, data.users, data.movies, num_negatives=16, batch_size=1024,
                          device=dev, seed=3)
    torch.manual_seed(1234)
    model = create_two_tower_model_for_training(3, 20, {"embedding_dim": 128, "hidden_layers": [256, 128],
                                                        "dropout_rate": 0.2, "temperature": 0.05}).to(dev)
    step = FusedTrainStep(model, lr=1e-3, weight_decay=1e-5, max_norm=1.0)
    fg = FeederGraph(step, feeder)
    fg.run_epoch(max_batches=8)  # capture + warm
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    losses = fg.run_epoch()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    nb = losses.numel()
    it = iter(feeder)

    def one():
        b = next(it)
        return step(b["user_table"], b["item_table"], b["item_table"], user_ids=b["user_ids"], pos_ids=b["pos_ids"],
                    neg_ids=b["neg_ids"])
    for _ in range(5):
        one()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(steps):
        one()
    torch.cuda.synchronize()
    el_eager = (time.perf_counter() - t1) / steps
    return {"ms_per_step": el / nb * 1e3, "pairs_per_s": (1024 * 1024 + 1024 * 16) * nb / el, "batches": nb,
            "epoch_s": el, "eager_ms_per_step": el_eager * 1e3,
            "note": "one epoch of FeederGraph replays (batch sampling: shuffle + on-device negatives inside the "
                    "graph, per-epoch permutation inside the timed region); eager_ms_per_step: the eager "
                    "feeder-iterated step"}


def c1_epoch(dev):
    """Config C1 (BASELINE.json configs[0]): one epoch of rtrec_amd.train_movielens
    at emb 64, batch 256, 16 negatives on the ML-1M-shaped stream (every train
    batch; feeder, fused steps, validation, checkpoint)."""
    import tempfile
    from rtrec_amd import train_movielens as tm
    with tempfile.TemporaryDirectory() as td:
        args = tm.build_parser().parse_args(["--synthetic", "--epochs", "1", "--batch-size", "256",
                                             "--embedding-dim", "64", "--checkpoint-dir", td + "/ckpt",
                                             "--output-dir", td + "/out", "--init-seed", "1234"])
        res = tm.run(args)
    n = res["batches_last_epoch"]
    return {"train_s": res["train_s"], "batches": n, "ms_per_batch": 1e3 * res["train_s"] / max(1, n),
            "pairs_per_s": n * (256 * 256 + 256 * 16) / res["train_s"], "train_loss": res["train_losses"][0],
            "val_loss": res["val_losses"][0],
            "note": "one full epoch incl. validation and checkpoint writes (reference CPU: ~33 ms/step at this "
                    "shape on the survey host, BASELINE.md §2)"}


# the csrc files each PMC-profiled kernel family is built from (its traffic
# figure is reused only while these are unchanged; tools/traffic_json.py)
# kernels whose fp32 products run on the bf16 MFMA through the three-piece split
SPLIT_BF16_KERNELS = ("linear_fwd", "linear_bwd_dz", "loss_fwd_bwd")
PEAK_BF16_TFLOPS = 2500.0  # dense bf16 MFMA, MI355X_MICROARCH.md

KERNEL_SOURCES = {
    "linear_fwd": ["mlp.hip", "split3.h", "rt_common.h"], "linear_bwd_dz": ["mlp.hip", "split3.h", "rt_common.h"],
    "linear_bwd_dw": ["mlp.hip", "split3.h", "rt_common.h"], "loss_fwd_bwd": ["loss.hip", "split3.h", "rt_common.h"],
    "clip_adam": ["optim.hip", "rt_common.h"], "gather_c5": ["gather.hip", "rt_common.h"],
    "flatip_topk_c4": ["topk_api.hip", "topk_f16.hip", "topk_impl.h", "topk_v1.h", "topk_v2.h", "topk_v3.h",
                       "topk_v4.h", "topk_dense.h", "rt_sort.h", "rt_common.h"],
}


def _kernel_sources_sha(kernel: str) -> str:
    import hashlib
    h = hashlib.sha256()
    csrc = os.path.join(PKG, "csrc")
    for f in sorted(KERNEL_SOURCES.get(kernel, [])):
        with open(os.path.join(csrc, f), "rb") as fh:
            h.update(f.encode() + b"\0" + fh.read())
    return h.hexdigest()[:16]


def pmc_traffic(kernel: str):
    """HBM bytes per launch of ``kernel`` from the newest profiles/*_traffic.json
    whose hash of that kernel's sources matches the sources being run
    (rocprofv3 FETCH_SIZE/WRITE_SIZE passes, tools/traffic_json.py); None if the
    PMC profile is older than the kernel."""
    import glob
    sha = _kernel_sources_sha(kernel)
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "*_traffic.json")), reverse=True):
        with open(path) as f:
            tj = json.load(f)
        shas = tj.get("kernel_sources_sha")
        if not isinstance(shas, dict) or shas.get(kernel) != sha:
            continue
        tb = tj.get("bytes_per_launch", {}).get(kernel)
        if tb is not None:
            return float(tb), f"{os.path.relpath(path, REPO)}: " + tj.get("correction", "")
    return None, f"no PMC profile of these {kernel} sources (sha {sha}) under profiles/"


def topk_c4_scaling(dev, dist, rank, world, reps=3):
    """C4 scaling leg, run collectively on every rank through the product
    index (rtrec_amd/serving/retrieval.py::HipShardedFlatIPIndex, the
    RetrievalEngine type "hip_flat_sharded"): a 1M-item f16 corpus (emb 128)
    row-sharded over the ranks (1M/N rows each, built rank-locally with
    build_shard), 65,536 queries per launch, k = 100, owner layout
    (search_tensors(layout="owner")). At N > 1 each launch is
    sharded_topk_global: every rank samples its shard, one all-gather of the
    sample lists' top r entries (bf16) gives one corpus-wide threshold per
    query, each rank searches its shard against it, one all-to-all sends the
    per-slice lists to the query owners, owner merge, then a device-summed
    count of short (rescue) queries read once on the host — the stage counts
    come from the shard sizes on the host (no collective). At N = 1 the index
    runs the plain single-GPU search. Strong scaling (fixed corpus);
    time = max over ranks between barriers."""
    from rtrec_amd.dist.sharded import LAST_TOPK, shard_range
    from rtrec_amd.serving.retrieval import HipShardedFlatIPIndex
    n, d, nq, k = 1_000_000, 128, 65536, 100
    b, c = shard_range(n, world, rank)
    g = torch.Generator(device=dev).manual_seed(1000 + rank)
    shard = torch.nn.functional.normalize(torch.randn(c, d, device=dev, generator=g), dim=1).half()
    gq = torch.Generator(device=dev).manual_seed(99)
    q = torch.nn.functional.normalize(torch.randn(nq, d, device=dev, generator=gq), dim=1).half()
    grp = dist.group.WORLD if dist is not None else None
    index = HipShardedFlatIPIndex({"dimension": d, "metric": "inner_product", "storage_dtype": "float16",
                                   "process_group": grp, "device": str(dev)})
    index.build_shard(shard, n, prepared=True)
    del shard

    def run():
        return index.search_tensors(q, k, layout="owner", prepared=True)

    def sync():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    run()
    sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        run()
    sync()
    el = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    del index, q
    torch.cuda.empty_cache()
    return {"qps": nq * reps / el, "ms_per_launch": 1e3 * el / reps, "n_gpus": world, "corpus_rows": n,
            "shard_rows": c, "queries_per_launch": nq, "k": k, "dtype": "f16",
            "api": "HipShardedFlatIPIndex.search_tensors(layout='owner') (RetrievalEngine 'hip_flat_sharded')",
            "exchange": ("sample lists all-gather (bf16 top-r), shard search against one corpus-wide threshold per "
                         "query, all_to_all + owner merge, rescue-count all-reduce (one host read)"
                         if world > 1 else "none (N = 1)"),
            "global_threshold": dict(LAST_TOPK) if world > 1 else None,
            "scaling": "strong (fixed 1M-row corpus)"}


def topk_c4_n8_emulated(dev, reps=3):
    """The per-rank work of the C4 1M-corpus search at N = 8, run on this one
    GPU (collectives excluded): (a) replicated corpus, 8,192 of the 65,536
    queries; (b) row shard 0 of 8 (125,000 rows) searched against one
    corpus-wide threshold per query — its sample, the threshold from the 8
    shards' sample lists (the other 7 precomputed, as the all-gather would
    deliver them), the shard search; (c) the same shard with its own
    threshold (the plain sharded search). Speed-up = the one-GPU 1M call over
    each per-rank time."""
    from rtrec_amd import kernels
    from rtrec_amd.dist.sharded import shard_range
    n, d, nq, k, world = 1_000_000, 128, 65536, 100, 8
    g = torch.Generator(device=dev).manual_seed(1000)
    corpus = torch.nn.functional.normalize(torch.randn(n, d, device=dev, generator=g), dim=1).half()
    gq = torch.Generator(device=dev).manual_seed(99)
    q = torch.nn.functional.normalize(torch.randn(nq, d, device=dev, generator=gq), dim=1).half()

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return 1e3 * (time.perf_counter() - t0) / reps
    t_full = timed(lambda: kernels.flatip_topk(q, corpus, k))
    mine = q[:nq // world].contiguous()
    t_repl = timed(lambda: kernels.flatip_topk(mine, corpus, k))
    b0, c0 = shard_range(n, world, 0)
    shard0 = corpus[b0:b0 + c0]
    stride = kernels.shard_sample_stride(n)
    lists, sampled, stages = [], 0, 0
    for r in range(world):
        b, c = shard_range(n, world, r)
        top, (sa, st) = kernels.flatip_topk_shard_sample(q, corpus[b:b + c], k, stride)
        lists.append(top)
        sampled += sa
        stages += st
    rank = kernels.topk_sample_rank(k, sampled, stages)
    stacked = torch.stack(lists)

    def rank_work():
        kernels.flatip_topk_shard_sample(q, shard0, k, stride)
        thr = kernels.topk_sample_threshold(stacked, rank)
        return kernels.flatip_topk_shard_search(q, shard0, k, thr, id_offset=b0)
    t_glob = timed(rank_work)
    _, ids = rank_work()
    cands = float((ids >= 0).sum(dim=1).float().mean())
    t_plain = timed(lambda: kernels.flatip_topk(q, shard0, k, id_offset=b0))
    del corpus, q, mine, stacked, lists
    torch.cuda.empty_cache()
    return {"one_gpu_1m_ms": t_full,
            "replicated_rank_ms": t_repl, "replicated_speedup": t_full / t_repl,
            "global_threshold_rank_ms": t_glob, "global_threshold_speedup": t_full / t_glob,
            "global_threshold_candidates_per_query": cands, "sample_rank": rank, "sample_stride": stride,
            "shard_local_threshold_rank_ms": t_plain, "shard_local_speedup": t_full / t_plain,
            "note": "per-rank device time at N = 8 on one GPU, collectives excluded (the driver's 8-GPU SCALE "
                    "run measures them)"}


def topk_c4_replicated(dev, dist, rank, world, reps=3):
    """C4 alternative layout, run collectively: the 1M-row f16 corpus (256 MB)
    REPLICATED on every GPU and the 65,536 queries of a launch split over the
    ranks (shard_range) — no exchange, no merge, each rank's lists final.
    Strong scaling on the same workload as topk_c4_1m_sharded; the row-sharded
    form keeps per-(query, shard) selection work that does not shrink with N."""
    from rtrec_amd import kernels
    from rtrec_amd.dist.sharded import shard_range
    n, d, nq, k = 1_000_000, 128, 65536, 100
    g = torch.Generator(device=dev).manual_seed(4242)  # same corpus on every rank
    corpus = torch.nn.functional.normalize(torch.randn(n, d, device=dev, generator=g), dim=1).half()
    gq = torch.Generator(device=dev).manual_seed(99)
    q = torch.nn.functional.normalize(torch.randn(nq, d, device=dev, generator=gq), dim=1).half()
    qb, qc = shard_range(nq, world, rank)
    mine = q[qb:qb + qc].contiguous()

    def sync():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    kernels.flatip_topk(mine, corpus, k)
    sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        kernels.flatip_topk(mine, corpus, k)
    sync()
    el = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    del corpus, q, mine
    torch.cuda.empty_cache()
    return {"qps": nq * reps / el, "ms_per_launch": 1e3 * el / reps, "n_gpus": world, "corpus_rows": n,
            "queries_per_rank": qc, "k": k, "dtype": "f16", "exchange": "none (corpus replicated, queries split)",
            "scaling": "strong (fixed 1M-row corpus, 65,536 queries per launch)"}


def c5_sharded_step(dev, dist, rank, world, reps=10):
    """C5 leg (SURVEY §8(e) training row), run collectively on every rank: a
    100M-row x 256 bf16 item table row-sharded 12.5M rows (6.4 GB) per GPU
    (weak scaling: the shard and the per-rank batch stay fixed as N grows, the
    table holds 12.5M·N rows), 8,192 users per rank with uniform global positive
    ids. One step = the row exchange (ids + row windows all-gather, each owner
    packs its positions' rows into a fixed segment, one all-gather of the
    segments; rtrec_amd/dist/sharded.py::sharded_gather_rows) +
    the 16-bit in-batch CE forward+backward of the rank's users against ALL
    gathered rows + the loss all-reduce (sharded_inbatch_step; the table is a
    frozen feature table as in the reference, so no item-gradient exchange). The
    same code runs at N = 1 (collectives skipped). time = max over ranks."""
    from rtrec_amd.dist.sharded import sharded_inbatch_step
    rows_per, dim, b, tau = 12_500_000, 256, 8192, 0.05
    g = torch.Generator(device=dev).manual_seed(2000 + rank)
    shard = torch.randn(rows_per, dim, device=dev, generator=g, dtype=torch.bfloat16) * 0.01
    row_begin = rank * rows_per
    gi = torch.Generator(device=dev).manual_seed(3000 + rank)
    ids = torch.randint(0, rows_per * world, (b,), device=dev, generator=gi)
    u = torch.nn.functional.normalize(torch.randn(b, dim, device=dev, generator=gi), dim=1).to(torch.bfloat16)
    grp = dist.group.WORLD if dist is not None else None

    def run():
        return sharded_inbatch_step(shard, row_begin, u, ids, tau, grp)

    def sync():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    run()
    sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        loss, _, _ = run()
    sync()
    el = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    from rtrec_amd.dist.sharded import LAST_EXCHANGE
    out = {"ms_per_step": 1e3 * el / reps, "n_gpus": world, "table_rows": rows_per * world, "shard_rows": rows_per,
           "emb_dim": dim, "users_per_rank": b, "dtype": "bf16", "loss": float(loss[0].item()),
           "pairs_per_s": world * b * (b * world) * reps / el,
           "exchange": ("ids + windows all-gather, owner-segment all-gather of rows (one host read of the "
                        "overflow flag), loss all-reduce" if world > 1 else "none (N = 1: collectives skipped)"),
           "exchange_mode": LAST_EXCHANGE.get("mode"), "segment_rows": LAST_EXCHANGE.get("segment_rows"),
           "bytes_exchanged_per_rank": LAST_EXCHANGE.get("bytes_per_rank", 0),
           "scaling": "weak (fixed shard and batch per GPU)"}
    del shard
    torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--no-extras", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--eager", action="store_true",
                    help="time eager steps (default: hipGraph replays of the captured step, inputs copied in)")
    args = ap.parse_args()
    # hipGraph replay (default): one graph per step on one GPU; under data
    # parallelism two graphs (gradients; clip+Adam) with the RCCL all-reduce of
    # the flat grad slab launched between them (FusedTrainStep.capture)
    args.graph = not args.eager

    dist, rank, world, dev = dist_setup(args.gpus)
    torch.cuda.set_device(dev)
    from rtrec_amd import native
    from rtrec_amd.profiling import TIMER
    from rtrec_amd.training.fused_step import FusedTrainStep
    native.lib()

    n_batches = min(args.steps + args.warmup, 64)
    model, (ut, mt), batches, host = c2_setup(dev, rank, n_batches)
    model.to(dev)
    step = FusedTrainStep(model, lr=1e-3, weight_decay=1e-5, max_norm=1.0,
                          process_group=(dist.group.WORLD if dist is not None else None))

    def run(i):
        bu, bp, bn = batches[i % n_batches]
        return step(ut, mt, mt, user_ids=bu, pos_ids=bp, neg_ids=bn)

    for i in range(args.warmup):
        run(i)
    # calibration step (eager, untimed): which ABI call dominates the step?
    # (a GPU spin before each call keeps host submission gaps out of the events)
    TIMER.enable(spacer_cycles=SPACER_CYCLES)
    run(args.warmup)
    cal = TIMER.summary()
    TIMER.disable()
    dominant = max(cal, key=lambda k: cal[k]["total_ms"])

    # timed region: eager steps, HIP events around every launch of the dominant
    # kernel on its launching stream (the roofline is measured live here).
    # --graph replays the whole step as a captured hipGraph instead (roofline then
    # from an eager pass right after).
    if args.graph:
        b0 = batches[0]
        st_pn = torch.cat([b0[1].reshape(-1), b0[2].reshape(-1)])  # adjacent static pos/neg ids
        st_ids = (b0[0].clone(), st_pn[:b0[1].numel()].view(b0[1].shape), st_pn[b0[1].numel():].view(b0[2].shape))
        try:
            step.capture(ut, mt, mt, user_ids=st_ids[0], pos_ids=st_ids[1], neg_ids=st_ids[2], warmup=1)
        except RuntimeError as e:  # no graph on this runtime: time eager steps instead
            log(f"hipGraph capture failed ({e}); timing eager steps")
            args.graph = False
    if args.graph:
        def run_timed(i):
            for dst, src in zip(st_ids, batches[i % n_batches]):
                dst.copy_(src, non_blocking=True)
            return step.replay()
    else:
        run_timed = run
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    if not args.graph:
        TIMER.enable([dominant])
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = run_timed(i)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if args.graph:
        TIMER.enable([dominant], spacer_cycles=SPACER_CYCLES)
        for i in range(args.steps):
            run(i)
    live = TIMER.summary()
    TIMER.disable()
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    final_loss = float(loss[0].item())

    pairs_per_step = 1024 * 1024 + 1024 * 16
    value = world * args.steps * pairs_per_step / elapsed
    d = live[dominant]
    per_launch_flops = d["flops"] / max(1, d["count"])
    per_launch_bytes = d["bytes"] / max(1, d["count"])
    avg_s = d["avg_ms"] * 1e-3
    if per_launch_flops > 0:
        achieved = per_launch_flops / avg_s / 1e12
        roof = {"bound": "mfma", "achieved": achieved, "peak": PEAK_F32_TFLOPS, "unit": "TFLOP/s",
                "frac": achieved / PEAK_F32_TFLOPS, "traffic": None}
    else:
        achieved = per_launch_bytes / avg_s / 1e9
        roof = {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": achieved / PEAK_HBM_GBS, "traffic": None}
    # HBM traffic per launch of the dominant kernel: rocprofv3 FETCH_SIZE / WRITE_SIZE
    # passes of this same bench command over the SAME kernel sources (else null)
    tb, tsrc = pmc_traffic(dominant)
    roof["traffic"] = tb
    roof["traffic_unit"] = "bytes/launch (PMC)"
    roof["traffic_source"] = tsrc
    if dominant in SPLIT_BF16_KERNELS:
        roof["peak_note"] = ("fp32-class products as 6 bf16 MFMAs each (three-piece split, DESIGN.md §5 note i): "
                             f"the instruction ceiling of this kernel is {PEAK_BF16_TFLOPS / 6:.0f} TFLOP/s "
                             f"(frac {achieved / (PEAK_BF16_TFLOPS / 6):.3f} of it); peak above = the fp32 MFMA")
    roof.update({"kernel": dominant, "launches_per_step": d["count"] / args.steps,
                 "measured": ("HIP events around each launch over an eager replay of the timed steps "
                              "(a GPU spin ahead of each launch keeps host submission out of the interval)"
                              if args.graph else "HIP events around each launch inside the timed region"),
                 "avg_launch_ms": d["avg_ms"], "step_share": cal[dominant]["total_ms"] /
                 max(1e-9, sum(v["total_ms"] for v in cal.values())),
                 "calibration_ms": {k: round(v["total_ms"], 4) for k, v in cal.items()}})

    result = {
        "metric": "user-item pairs scored/sec (train) + top-K queries/sec, emb_dim=128",
        "value": value, "unit": "pairs/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": 1000.0 * elapsed / args.steps, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "vs_baseline_source": (
            f"BASELINE.md §2: the reference's own CPU C2 step, {BASELINE_MD_C2_MS:g} ms = "
            f"{BASELINE_MD_C2_PAIRS_PER_S / 1e6:.2f} M pairs/s (survey container, 8 ATen threads; a different "
            f"machine from this run: vs_cpu_baseline_same_box divides by cpu_baseline.value measured here)"),
        "dtype": "f32",
        "data": "synthetic ML-1M-shaped (6040 users x 3416 movies, seeded; ratings.dat unavailable)",
        "config": {"workload": "C2: MovieLens-1M two-tower train step, emb 128, batch 1024, 16 negatives, "
                               "hidden [256,128], dropout 0.2, tau 0.05, Adam+clip",
                   "global_batch": 1024 * world, "emb_dim": 128, "num_negatives": 16,
                   "parallelism": f"dp{world}", "final_loss": final_loss},
        "roofline": roof,
    }
    result["vs_baseline"] = value / BASELINE_MD_C2_PAIRS_PER_S
    scaling = c5 = repl = None
    if not args.no_extras:  # collective: every rank
        try:
            scaling = topk_c4_scaling(dev, dist, rank, world)
        except Exception as e:  # extras never hide the headline
            scaling = {"error": repr(e)}
        try:
            c5 = c5_sharded_step(dev, dist, rank, world)
        except Exception as e:
            c5 = {"error": repr(e)}
        try:
            repl = topk_c4_replicated(dev, dist, rank, world)
        except Exception as e:
            repl = {"error": repr(e)}
    if rank == 0 and world == 1:
        if not args.no_extras:
            try:
                result["extras"] = topk_extras(dev)
            except Exception as e:  # extras never hide the headline
                result["extras"] = {"error": repr(e)}
            legs = [("c2_with_feeder", lambda: c2_with_feeder(dev)), ("c1_train_epoch", lambda: c1_epoch(dev))]
            if world == 1:
                legs.append(("topk_c4_n8_emulated", lambda: topk_c4_n8_emulated(dev)))
            for name, fn in legs:
                try:
                    result["extras"][name] = fn()
                except Exception as e:
                    result["extras"][name] = {"error": repr(e)}
        if not args.no_cpu_baseline:
            result["cpu_baseline"] = cpu_baseline(host, args.cpu_budget)
            # two ratios, two machines: vs_baseline (the headline field) divides by
            # BASELINE.md's reference step timed in the survey container; this one
            # divides by the oracle step timed on THIS box's host cores in this run
            result["vs_cpu_baseline_same_box"] = value / result["cpu_baseline"]["value"]
            if _cpu_cores() < _host_cores():
                result["cpu_baseline"]["note"] = (
                    f"threads = the {_cpu_cores()} CPUs of this process's cgroup quota, not the "
                    f"{_host_cores()}-core affinity set: {_host_cores()} threads on a {_cpu_cores()}-CPU quota "
                    "oversubscribe it (r03s1: 30.7 s for one step)")
            try:
                result["cpu_baseline"]["topk"] = cpu_topk_baseline()
                ex = result.get("extras", {})
                if "topk_c3" in ex and "qps" in ex["topk_c3"]:
                    ex["topk_c3"]["vs_cpu"] = ex["topk_c3"]["qps"] / result["cpu_baseline"]["topk"]["topk_c3"]["qps"]
            except Exception as e:
                result["cpu_baseline"]["topk"] = {"error": repr(e)}
    if c5 is not None:
        result.setdefault("extras", {})["c5_sharded_step"] = c5
    if repl is not None:
        result.setdefault("extras", {})["topk_c4_1m_replicated"] = repl
    if scaling is not None:
        result.setdefault("extras", {})["topk_c4_1m_sharded"] = scaling
        cb = result.get("cpu_baseline", {}).get("topk", {}).get("topk_c4")
        if cb and "qps" in scaling:
            scaling["vs_cpu"] = scaling["qps"] / cb["qps"]
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
