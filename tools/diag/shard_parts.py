"""Times the parts of the C4 N = 8 per-rank work (sample of shard 0, the
corpus-wide threshold, the shard search) and the plain 1M / 8K-query calls,
for the library RTREC_HIP_LIB points at. Prints one JSON line."""
import json
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
thr = kernels.topk_sample_threshold(stacked, rank)


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return [round(1e3 * (time.perf_counter() - t0) / reps, 3), round(e0.elapsed_time(e1) / reps, 3)]


out = {"lib": os.path.basename(os.environ.get("RTREC_HIP_LIB", "default"))}
out["sample"] = timed(lambda: kernels.flatip_topk_shard_sample(q, shard0, k, stride))
out["threshold"] = timed(lambda: kernels.topk_sample_threshold(stacked, rank))
out["search"] = timed(lambda: kernels.flatip_topk_shard_search(q, shard0, k, thr, id_offset=b0))
out["plain_125k"] = timed(lambda: kernels.flatip_topk(q, shard0, k))
mine = q[:nq // world].contiguous()
out["q8k_1m"] = timed(lambda: kernels.flatip_topk(mine, corpus, k))
out["full_1m"] = timed(lambda: kernels.flatip_topk(q, corpus, k), reps=2)
print(json.dumps(out), flush=True)
