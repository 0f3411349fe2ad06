"""Multi-process GPU check of HipShardedFlatIPIndex (RetrievalEngine index_type
"hip_flat_sharded"), run as one rank per process under torch.distributed.run:

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port P tools/sharded_index_ranks.py OUT_JSON

Every rank uses cuda:0 with the gloo backend (RCCL refuses two ranks on one
device; on a multi-GPU node the same code runs one rank per GPU over RCCL), so
the HIP kernels of the corpus-wide-threshold search (shard sample, threshold,
shard search, merge) run for real with the exchange steps in between. The
corpus is dyadic f16 (every fp32 partial sum exact, so any kernel's order
gives the same bits) with planted exact ties; each rank compares the sharded
engine with one whole-corpus HipFlatIPIndex of the same rows id for id and
score for score: plain search, filter_ids, add (rows spread over the ranks),
and a forced rescue. tests/test_gpu_dist.py launches it."""
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist


def main(out_path):
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from rtrec_amd.dist import sharded as sh
    from rtrec_amd.serving.retrieval import HipFlatIPIndex, RetrievalEngine
    rng = np.random.default_rng(17)
    n, d, nq, k = 65_536 * world + 4099, 128, 8192, 100  # >= 7,681 queries: the v4 plan
    corpus = (rng.integers(-8, 9, size=(n, d)) / 64.0).astype(np.float32)
    corpus[n - 1] = corpus[5]
    corpus[n // 2 + 1] = corpus[7]
    queries = (rng.integers(-8, 9, size=(nq, d)) / 64.0).astype(np.float32)
    ids = [f"m{p}" for p in range(n)]
    cfg = {"index_type": "hip_flat_sharded", "embedding_dim": d, "top_k": k,
           "hip_flat_sharded": {"metric": "inner_product", "storage_dtype": "float16", "device": str(dev)}}
    eng = RetrievalEngine(cfg)
    eng.build_index(corpus, ids)
    flat = HipFlatIPIndex({"dimension": d, "metric": "inner_product", "storage_dtype": "float16",
                           "device": str(dev)})
    flat.build(corpus, ids)
    report = {"rank": rank, "world": world, "checks": []}

    def check(name, q, kk, filt=None):
        got = eng.retrieve(q, kk, filt, use_cache=False)[:2]
        want = flat.search(q, kk, filt)
        ok = got == want
        report["checks"].append({"name": name, "ok": ok, "path": dict(sh.LAST_TOPK)})
        if not ok:
            bad = [i for i in range(len(want[0])) if got[0][i] != want[0][i]]
            report["checks"][-1]["first_bad_query"] = bad[:3]
        return ok

    check("search k=100", queries, k)
    check("search k=10", queries[:777], 10)
    check("filter_ids", queries, 20, ids[::4])        # k_search 40: the global path
    check("filter_ids small batch", queries[:300], 20, ids[::4])
    extra = (rng.integers(-8, 9, size=(3001, d)) / 64.0).astype(np.float32)
    extra[0] = corpus[5]
    eng.update_index(extra, [f"x{j}" for j in range(3001)])
    flat.add(extra, [f"x{j}" for j in range(3001)])
    check("after add", queries, k)
    # owner layout equals the all-gather layout's slice
    q16 = torch.from_numpy(queries).to(dev).half()
    so, po = eng.index.search_tensors(q16, k, layout="owner", prepared=True)
    sa, pa = eng.index.search_tensors(q16, k, prepared=True)
    per = nq // world
    report["checks"].append({"name": "owner slice", "ok": bool(torch.equal(po, pa[rank * per:(rank + 1) * per])
                                                               and torch.equal(so, sa[rank * per:(rank + 1) * per]))})
    # forced rescue: an unsafe sample rank (threshold above the k-th) must still be exact
    real = eng.index._ops

    def forced(rows):
        ops = real(rows)
        ops.rank = lambda kk, s, t: 1
        return ops
    eng.index._ops = forced
    check("forced rescue", queries, k)
    eng.index._ops = real
    report["ok"] = all(c["ok"] for c in report["checks"])
    with open(f"{out_path}.rank{rank}", "w") as f:
        json.dump(report, f, indent=1)
    dist.barrier()
    dist.destroy_process_group()
    return 0 if report["ok"] else 1


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
