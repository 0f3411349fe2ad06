#!/usr/bin/env python3
"""Per-step device times of the N = 8 global-threshold C4 rank work on one GPU
(bench.topk_c4_n8_emulated's shard 0): the shard sample, the threshold combine
of 8 shards' lists, the shard search (scan against the threshold + finish),
next to the plain shard search and the replicated 8,192-query slice. HIP-event
timed, 5 reps each after a warmup.  Usage: python tools/prof_shard_modes.py"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "real-time-recommendation-system-with-feature-store_amd")]

import torch  # noqa: E402

from rtrec_amd import kernels  # noqa: E402
from rtrec_amd.dist.sharded import shard_range  # noqa: E402


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    dev = torch.device("cuda", 0)
    n, d, nq, k, world = 1_000_000, 128, 65536, 100, 8
    g = torch.Generator(device=dev).manual_seed(1000)
    corpus = torch.nn.functional.normalize(torch.randn(n, d, device=dev, generator=g), dim=1).half()
    gq = torch.Generator(device=dev).manual_seed(99)
    q = torch.nn.functional.normalize(torch.randn(nq, d, device=dev, generator=gq), dim=1).half()
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
    b0, c0 = shard_range(n, world, 0)
    shard0 = corpus[b0:b0 + c0]
    thr = kernels.topk_sample_threshold(stacked, rank)
    out = {
        "sample_ms": timed(lambda: kernels.flatip_topk_shard_sample(q, shard0, k, stride)),
        "threshold_ms": timed(lambda: kernels.topk_sample_threshold(stacked, rank)),
        "search_ms": timed(lambda: kernels.flatip_topk_shard_search(q, shard0, k, thr, id_offset=b0)),
        "plain_shard_ms": timed(lambda: kernels.flatip_topk(q, shard0, k, id_offset=b0)),
        "replicated_slice_ms": timed(lambda: kernels.flatip_topk(q[:nq // world].contiguous(), corpus, k)),
        "stride": stride, "rank": rank,
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
