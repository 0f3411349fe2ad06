"""GPU side of the multi-GPU paths, in one process: the per-rank kernels of
the corpus-sharded top-K (rt_flatip_topk with a shard id offset, then
rt_topk_merge over the stacked per-shard lists, exactly what every rank runs
after its all_gather) must reproduce one unsharded search bit-exactly; the
table-window gather must equal the unsharded gather after the sum."""
import numpy as np
import pytest
import torch

from oracle import flat_ip as orc
from rtrec_amd import kernels
from rtrec_amd.dist.sharded import ShardedFlatIPIndex, shard_range

pytestmark = pytest.mark.gpu


def _dyadic(rng, n, d):
    return (rng.integers(-64, 65, size=(n, d)) / 64.0).astype(np.float32)


@pytest.mark.parametrize("world,n,k,dtype", [(2, 1001, 10, torch.float32), (8, 5000, 100, torch.float32),
                                             (8, 4096, 100, torch.float16), (3, 97, 50, torch.bfloat16)])
def test_shard_then_merge_equals_single_search(device, world, n, k, dtype):
    rng = np.random.default_rng(11)
    d = 128
    corpus = _dyadic(rng, n, d)
    corpus[-1] = corpus[0]      # exact ties across shards: lower global id wins
    queries = _dyadic(rng, 67, d)
    q = torch.from_numpy(queries).to(device, dtype)
    x = torch.from_numpy(corpus).to(device, dtype)
    lists_s, lists_i = [], []
    for r in range(world):
        b, c = shard_range(n, world, r)
        s, i = kernels.flatip_topk(q, x[b:b + c], k, id_offset=b)
        lists_s.append(s)
        lists_i.append(i)
    ms, mi = kernels.topk_merge(torch.stack(lists_s), torch.stack(lists_i), k)
    fs, fi = kernels.flatip_topk(q, x, k)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(mi.cpu().numpy(), fi.cpu().numpy())
    np.testing.assert_array_equal(ms.cpu().numpy(), fs.cpu().numpy())
    if dtype == torch.float32:   # and both equal the oracle (Faiss restatement)
        rs, ri = orc.flat_ip_search(queries, corpus, k)
        np.testing.assert_array_equal(mi.cpu().numpy(), ri)
        np.testing.assert_array_equal(ms.cpu().numpy(), rs)


def test_sharded_index_single_rank_matches_flat_index(device):
    from rtrec_amd.serving.retrieval import HipFlatIPIndex
    rng = np.random.default_rng(5)
    corpus = rng.standard_normal((3000, 64)).astype(np.float32)
    queries = rng.standard_normal((40, 64)).astype(np.float32)
    sh = ShardedFlatIPIndex(64, device=device).build(corpus)
    flat = HipFlatIPIndex({"dimension": 64, "metric": "cosine", "device": str(device)})
    flat.build(corpus, [str(i) for i in range(len(corpus))])
    s1, i1 = sh.search_tensors(queries, 20)
    s2, i2 = flat.search_tensors(queries, 20)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(i1.cpu().numpy(), i2.cpu().numpy())
    np.testing.assert_array_equal(s1.cpu().numpy(), s2.cpu().numpy())
    # excluded global ids never come back
    ex = [list(i1[q, :5].cpu().numpy()) for q in range(40)]
    s3, i3 = sh.search_tensors(queries, 20, excluded=ex)
    got = i3.cpu().numpy()
    for q in range(40):
        assert not set(ex[q]) & set(got[q].tolist())
        np.testing.assert_array_equal(got[q, :15], i1[q, 5:].cpu().numpy())


def test_table_window_gather_sums_to_full_gather(device):
    rng = np.random.default_rng(2)
    n, d, world = 1003, 256, 4
    table = torch.from_numpy(rng.standard_normal((n, d)).astype(np.float32)).to(device, torch.bfloat16)
    ids = torch.from_numpy(rng.integers(0, n, size=517)).to(device)
    acc = torch.zeros((517, d), dtype=torch.float32, device=device)
    for r in range(world):
        b, c = shard_range(n, world, r)
        acc += kernels.gather_rows(table[b:b + c], ids, row_begin=b).float()
    ref = kernels.gather_rows(table, ids).float()
    torch.cuda.synchronize()
    assert torch.equal(acc, ref)
    assert torch.equal(ref, table[ids].float())
