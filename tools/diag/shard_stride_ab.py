"""Per-rank device time of the C4 sharded search at N = 8 (bench.py
topk_c4_n8_emulated (b): shard 0 of a 1M-row corpus, its sample, the
corpus-wide threshold from all 8 shards' lists, the shard search) for several
sample strides, interleaved. Usage: python tools/diag/shard_stride_ab.py [ROUNDS]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..",
                                "real-time-recommendation-system-with-feature-store_amd"))
from rtrec_amd import kernels  # noqa: E402
from rtrec_amd.dist.sharded import shard_range  # noqa: E402

n, d, nq, k, world = 1_000_000, 128, 65536, 100, 8
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(1000)
corpus = torch.nn.functional.normalize(torch.randn(n, d, device=dev, generator=g), dim=1).half()
gq = torch.Generator(device=dev).manual_seed(99)
q = torch.nn.functional.normalize(torch.randn(nq, d, device=dev, generator=gq), dim=1).half()
b0, c0 = shard_range(n, world, 0)
shard0 = corpus[b0:b0 + c0]


def setup(stride):
    lists, sampled, stages = [], 0, 0
    for r in range(world):
        b, c = shard_range(n, world, r)
        top, (sa, st) = kernels.flatip_topk_shard_sample(q, corpus[b:b + c], k, stride)
        lists.append(top)
        sampled += sa
        stages += st
    rank = kernels.topk_sample_rank(k, sampled, stages)
    stacked = torch.stack(lists)

    def work():
        kernels.flatip_topk_shard_sample(q, shard0, k, stride)
        thr = kernels.topk_sample_threshold(stacked, rank)
        return kernels.flatip_topk_shard_search(q, shard0, k, thr, id_offset=b0)
    return rank, work


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t0) / reps


ref = None
works = {}
for st in (64, 32, 16):
    rank, w = setup(st)
    s, i = w()
    if ref is None:
        ref = (s.clone(), i.clone())
    same = bool(torch.equal(i, ref[1]) and torch.equal(s, ref[0]))
    works[st] = w
    print(f"stride {st}: rank {rank}, candidates/query {float((i >= 0).sum(1).float().mean()):.1f}, "
          f"same output as stride 64: {same}", flush=True)
for r in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    print(" ".join(f"s{st} {timed(w):.3f}" for st, w in works.items()), flush=True)
