"""Row-sharded lookup exchange (recommender_system_amd/sharded.py).

CPU, world_size 2 and 3 over gloo: the all-to-all protocol returns exactly the
rows of the global table for every lookup, and the FM on them equals the
oracle on the unsharded model.  The per-rank local steps use a numpy test
double (CpuOps) here; on the GPU they are the HIP kernels, whose bucketize /
gather / unpermute are checked against the same double in the gpu test below.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import ctr_oracle as O


class CpuOps:
    """numpy restatement of the per-rank steps (test double, not product code)."""

    def bucketize(self, ids, offsets, vocab, rpr, world):
        ids_n = ids.numpy().astype(np.int64)
        rows = offsets.numpy()[None, :] + ids_n
        owner = np.minimum(rows // rpr, world - 1).reshape(-1)
        order = np.argsort(owner, kind="stable")
        perm = np.empty_like(order)
        perm[order] = np.arange(order.size)
        send = np.empty(order.size, np.int64)
        send[perm] = rows.reshape(-1) - owner * rpr
        counts = np.bincount(owner, minlength=world)
        return (torch.as_tensor(counts, dtype=torch.int32), torch.as_tensor(perm, dtype=torch.int32),
                torch.as_tensor(send, dtype=torch.int32))

    def __init__(self):
        self.overflow = False

    def slot_bucketize(self, ids, offsets, vocab, rpr, world, cap, bufs=None):
        """Fixed-capacity slots: lookup j of owner o with stable rank r < cap
        goes to slot o*cap + r; unused slots ask for row -1."""
        ids_n = ids.numpy().astype(np.int64)
        rows = (offsets.numpy()[None, :] + ids_n).reshape(-1)
        owner = np.minimum(rows // rpr, world - 1)
        slot_of = np.full(rows.size, -1, np.int64)
        send = np.full(world * cap, -1, np.int64)
        for o in range(world):
            idx = np.nonzero(owner == o)[0]  # stable (ascending lookup order)
            if idx.size > cap:
                self.overflow = True
            idx = idx[:cap]
            slot_of[idx] = o * cap + np.arange(idx.size)
            send[o * cap + np.arange(idx.size)] = rows[idx] - o * rpr
        return torch.as_tensor(slot_of, dtype=torch.int32), torch.as_tensor(send, dtype=torch.int32)

    def gather_rows_into(self, table, rows, out=None):
        r = rows.long()
        got = table[r.clamp(min=0)]
        got[r < 0] = 0
        return got

    def slots_fm(self, got, slot_of, dense, F, k, prepared, w0, kfm, bufs=None, out=None):
        self.last_emb = got[slot_of.long()]
        return None

    def flags(self, bufs=None):
        f = torch.tensor([0, int(self.overflow)], dtype=torch.int32)
        self.overflow = False
        return f

    def gather_rows(self, table, rows):
        return table[rows.long()]

    def unpermute(self, src, perm):
        return src[perm.long()]

    def rows_fm(self, emb, dense, F, k, prepared, w0, kfm):
        self.last_emb = emb
        return None


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, vocabs, k, B, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from recommender_system_amd.sharded import ShardedEmbeddingFM
        ops = CpuOps()
        sh = ShardedEmbeddingFM(vocabs, k, nd=3, kfm=4, device="cpu", seed=7, ops=ops)
        rng = np.random.default_rng(100 + rank)
        ids = torch.as_tensor(np.stack([rng.integers(0, v, B) for v in vocabs], 1), dtype=torch.int32)
        emb = sh.lookup(ids)
        # reference: the full table assembled from every rank's shard
        shards = [None] * world
        dist.all_gather_object(shards, sh.table_shard.numpy())
        full = np.concatenate(shards)
        rows = sh.offsets.numpy()[None, :] + ids.numpy()
        expect = full[rows.reshape(-1)]
        ok_rows = np.array_equal(emb.numpy(), expect)
        # fixed-capacity exchange: same rows through the slots
        got, slot_of = sh.exchange_slots(ids)
        ok_rows = ok_rows and np.array_equal(got[slot_of.long()].numpy(), expect)
        # forced overflow (tiny capacity on every rank): forward() falls back to
        # the exact protocol, collectively, and still returns the exact rows
        sh._slot_bufs = None
        sh.capacity = lambda n: 2
        dense0 = torch.zeros(B, 3)
        sh.forward(dense0, ids)
        ok_rows = ok_rows and np.array_equal(ops.last_emb.numpy(), expect)
        dense = rng.random((B, 3)).astype(np.float32)
        x = np.concatenate([dense, emb.numpy().reshape(B, -1)], 1)
        fm_sh = O.fm_layer(x, sh.w0.numpy(), sh.w1.numpy(), sh.v.numpy())
        tables = [full[o:o + v] for o, v in zip(sh.offsets.numpy(), vocabs)]
        fm_ref = O.deepfm(None, {"tables": tables, "w0": sh.w0.numpy(), "w1": sh.w1.numpy(), "v": sh.v.numpy(),
                                 "dnn_hidden": [], "dnn_out": (np.zeros((x.shape[1], 1)), np.zeros(1))},
                          nd=3, inputs=(dense, ids.numpy()))[1]
        q.put((rank, ok_rows, float(np.max(np.abs(fm_sh - fm_ref))), sh.row_range))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_exchange_gloo(world):
    vocabs = [50, 7, 300, 1, 120]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, vocabs, 4, 33, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    ranges = [r[3] for r in res]
    assert ranges[0][0] == 0 and ranges[-1][1] == sum(vocabs)
    assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))
    for rank, ok_rows, fm_err, _ in res:
        assert ok_rows, f"rank {rank}: exchanged rows differ from the global table"
        assert fm_err < 1e-12


@pytest.mark.gpu
@pytest.mark.parametrize("world", [1, 3, 8])
def test_gpu_shard_kernels_match_reference(gpu, world):
    from recommender_system_amd.sharded import HipShardOps
    rng = np.random.default_rng(world)
    vocabs = rng.integers(1, 5000, 26)
    offs = np.concatenate([[0], np.cumsum(vocabs)[:-1]])
    B = 1000
    ids = np.stack([rng.integers(0, v, B) for v in vocabs], 1)
    rpr = int(np.ceil(vocabs.sum() / world))
    ops = HipShardOps(gpu)
    c, p, s = ops.bucketize(torch.as_tensor(ids, dtype=torch.int32, device=gpu),
                            torch.as_tensor(offs, device=gpu), torch.as_tensor(vocabs, device=gpu), rpr, world)
    rc, rp, rs_ = CpuOps().bucketize(torch.as_tensor(ids), torch.as_tensor(offs), None, rpr, world)
    np.testing.assert_array_equal(c.cpu().numpy(), rc.numpy())
    np.testing.assert_array_equal(p.cpu().numpy(), rp.numpy())
    np.testing.assert_array_equal(s.cpu().numpy(), rs_.numpy())
    table = torch.randn(int(vocabs.sum()), 16, device=gpu)
    rows = torch.as_tensor(rng.integers(0, table.shape[0], 777), dtype=torch.int32, device=gpu)
    np.testing.assert_array_equal(ops.gather_rows(table, rows).cpu().numpy(), table[rows.long()].cpu().numpy())
    src = torch.randn(B * 26, 16, device=gpu)
    np.testing.assert_array_equal(ops.unpermute(src, p).cpu().numpy(), src[p.long()].cpu().numpy())
    ops.check()


@pytest.mark.gpu
def test_gpu_sharded_single_rank_equals_fused(gpu):
    """world=1 exchange path (bucketize -> gather -> unpermute -> rows FM)
    equals the fused kernel on the same table."""
    from recommender_system_amd import _lib
    from recommender_system_amd.sharded import ShardedEmbeddingFM
    vocabs = [1000, 50, 3000, 7] * 6 + [11, 12]
    sh = ShardedEmbeddingFM(vocabs, 16, 13, 10, device=gpu, seed=3)
    rng = np.random.default_rng(0)
    B = 300
    ids = torch.as_tensor(np.stack([rng.integers(0, v, B) for v in vocabs], 1), dtype=torch.int32, device=gpu)
    dense = torch.rand(B, 13, device=gpu)
    a = sh.forward(dense, ids)                 # fixed-capacity slots (default)
    e = sh.forward_exact(dense, ids)           # counts + variable splits
    sh._slot_bufs = None
    sh.capacity = lambda n: 7                  # forced overflow -> exact fallback
    f = sh.forward(dense, ids)
    b = torch.empty(B, 1, device=gpu)
    _lib.call("rs_embed_fm_fwd", ids.data_ptr(), 0, 26, dense.data_ptr(), 13, 13, sh.table_shard.data_ptr(),
              sh.offsets.data_ptr(), sh.vocab.data_ptr(), 26, 16, sh.prepared.data_ptr(), sh.w0.data_ptr(), 10,
              b.data_ptr(), None, B, None, _lib.stream())
    np.testing.assert_allclose(a.cpu().numpy(), b.cpu().numpy(), rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(e.cpu().numpy(), b.cpu().numpy(), rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(f.cpu().numpy(), b.cpu().numpy(), rtol=1e-6, atol=1e-6)
    bad = ids.clone()
    bad[3, 5] = vocabs[5]
    sh.capacity = lambda n: max(n, 1)
    sh._slot_bufs = None
    with pytest.raises(IndexError):
        sh.forward(dense, bad)


@pytest.mark.gpu
@pytest.mark.parametrize("world,cap", [(1, 26000), (3, 3000), (8, 1100), (8, 900)])
def test_gpu_slot_bucketize_matches_reference(gpu, world, cap):
    """rs_shard_slot_bucketize == the numpy slot double (incl. overflow)."""
    from recommender_system_amd.sharded import HipShardOps
    rng = np.random.default_rng(world + cap)
    vocabs = rng.integers(1, 5000, 26)
    offs = np.concatenate([[0], np.cumsum(vocabs)[:-1]])
    B = 1000
    ids = np.stack([rng.integers(0, v, B) for v in vocabs], 1)
    rpr = int(np.ceil(vocabs.sum() / world))
    ops = HipShardOps(gpu)
    bufs = {"counts": torch.empty(world, dtype=torch.int32, device=gpu),
            "slot_of": torch.empty(B * 26, dtype=torch.int32, device=gpu),
            "send": torch.full((world * cap,), -1, dtype=torch.int32, device=gpu),
            "overflow": torch.zeros(1, dtype=torch.int32, device=gpu)}
    so, send = ops.slot_bucketize(torch.as_tensor(ids, dtype=torch.int32, device=gpu), torch.as_tensor(offs, device=gpu),
                                  torch.as_tensor(vocabs, device=gpu), rpr, world, cap, bufs)
    ref = CpuOps()
    rso, rsend = ref.slot_bucketize(torch.as_tensor(ids), torch.as_tensor(offs), None, rpr, world, cap)
    np.testing.assert_array_equal(so.cpu().numpy(), rso.numpy())
    np.testing.assert_array_equal(send.cpu().numpy(), rsend.numpy())
    assert bool(bufs["overflow"].item()) == ref.overflow
