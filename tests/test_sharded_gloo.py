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

    # row protocol of ShardedDeepFM
    def row_route(self, sh, ids, send, slot_of):
        ids_n = ids.numpy().astype(np.int64)
        B, F = ids_n.shape
        S = sh.slot_stride
        out = np.full((sh.world, B, S), -1, np.int64)
        slot = np.full((B, F), -1, np.int64)
        rows = sh.offsets.numpy()[None, :] + ids_n
        for o, (lo, n) in enumerate(sh.owner_field_ranges):
            for j in range(n):
                loc = rows[:, lo + j] - o * sh.rows_per_rank
                m = (loc >= 0) & (loc < sh.rows_per_rank)
                out[o, m, j] = loc[m]
                slot[m, lo + j] = (o * B + np.nonzero(m)[0]) * S + j
        send.copy_(torch.as_tensor(out.reshape(-1), dtype=torch.int32))
        slot_of.copy_(torch.as_tensor(slot, dtype=torch.int32))
        return send, slot_of

    def deepfm_rows(self, model, got, rb, dense, out):
        so = rb["slot_of"].numpy().astype(np.int64)
        emb = got.numpy().astype(np.float64)[so]  # [B, F, k]
        self.last_emb = emb.reshape(-1, emb.shape[-1])
        x = np.concatenate([np.asarray(dense, np.float64), emb.reshape(so.shape[0], -1)], 1)
        c = lambda t: t.detach().numpy()
        hidden = [(c(l.kernel), c(l.bias)) for l in model.dnn.hidden_layer]
        o = model.dnn.output_layer
        fm = O.fm_layer(x, c(model.emb.w0), c(model.emb.w1), c(model.emb.v))
        dnn = O.dnn_layer(x, hidden, (c(o.kernel), c(o.bias)))
        out.copy_(torch.as_tensor(O.sigmoid(0.5 * (fm + dnn)), dtype=torch.float32))
        return out

    # dedup exchange of ShardedDeepFM
    def dedup_route(self, sh, ids, rb):
        ids_n = ids.numpy().astype(np.int64)
        B, F = ids_n.shape
        cap = rb["cap"]
        rows = (sh.offsets.cpu().numpy()[None, :] + ids_n).reshape(-1)
        owner = np.minimum(rows // sh.rows_per_rank, sh.world - 1)
        send = np.full(sh.world * cap, -1, np.int64)
        slot = np.full(rows.size, -1, np.int64)
        for o in range(sh.world):
            u, inv = np.unique(rows[owner == o], return_inverse=True)
            if u.size > cap:
                self.dedup_overflow = True
            keep = inv < cap
            idx = np.nonzero(owner == o)[0]
            slot[idx[keep]] = o * cap + inv[keep]
            send[o * cap + np.arange(min(u.size, cap))] = u[:cap] - o * sh.rows_per_rank
        rb["send"].copy_(torch.as_tensor(send, dtype=torch.int32))
        rb["slot_of"].copy_(torch.as_tensor(slot.reshape(B, F), dtype=torch.int32))
        return rb["send"], rb["slot_of"]

    def overflow_flag(self, rb):
        f = torch.tensor([int(getattr(self, "dedup_overflow", False))], dtype=torch.int32)
        self.fallbacks = getattr(self, "fallbacks", 0) + int(f.item())
        self.dedup_overflow = False
        return f

    def dedup_grads(self, model, dx, rb):
        so = rb["slot_of"].numpy().reshape(-1).astype(np.int64)
        rows = dx.numpy()[:, model.nd:].reshape(-1, model.k).astype(np.float64)
        acc = np.zeros((rb["n"], model.k))
        np.add.at(acc, so[so >= 0], rows[so >= 0])
        g = rb["gsend"].numpy()
        used = np.unique(so[so >= 0])
        g[used] = acc[used]
        return rb["gsend"]

    # training of ShardedDeepFM (fp64 inside, fp32 buffers like the device path)
    def deepfm_grads(self, model, got, rb, dense, labels, scale, tb, loss, drop=None):
        so = rb["slot_of"].numpy().astype(np.int64)
        B = so.shape[0]
        x = np.concatenate([np.asarray(dense, np.float64), got.numpy().astype(np.float64)[so].reshape(B, -1)], 1)
        c = lambda t: t.detach().numpy().astype(np.float64)
        sh = model.emb
        layers = [(c(l.kernel), c(l.bias)) for l in model.dnn.hidden_layer]
        layers.append((c(model.dnn.output_layer.kernel), c(model.dnn.output_layer.bias)))
        masks = None
        if drop is not None:  # the rank's draws, restated by the oracle's generator
            rng, rate, offs = drop
            base = int(rng.base.item())  # offsets are relative to the generator's counter
            masks = [O.dropout_multiplier(B, W_.shape[1], rate, rng.seed, base + o)
                     for (W_, _), o in zip(layers, offs)]
            rng.base += rng.rel  # end of the step (models._Dropout.end_step, on the host here)
            rng.rel = 0
        acts = [x]
        for i, (W_, b_) in enumerate(layers[:-1]):
            a = np.maximum(acts[-1] @ W_ + b_, 0.0)
            acts.append(a * masks[i] if masks is not None else a)
        dnn = (acts[-1] @ layers[-1][0] + layers[-1][1])[:, 0]
        w0, w1, v = c(sh.w0), c(sh.w1), c(sh.v)
        z = 0.5 * (O.fm_layer(x, w0, w1, v)[:, 0] + dnn)
        t = labels.numpy().astype(np.float64)
        if loss is not None:
            loss.copy_(torch.as_tensor(np.maximum(z, 0) - z * t + np.log1p(np.exp(-np.abs(z)))))
        gf = 0.5 * scale * (O.sigmoid(z) - t)
        delta = gf[:, None]
        for li in reversed(range(len(layers))):
            dW, db = tb["dnn_views"][li]
            dW.copy_(torch.as_tensor(acts[li].T @ delta))
            db.copy_(torch.as_tensor(delta.sum(0)))
            prev = delta @ layers[li][0].T
            if li > 0:
                prev = prev * (acts[li] > 0)
                if masks is not None:
                    prev = prev * masks[li - 1]
            delta = prev
        s = x @ v
        dx = delta + gf[:, None] * (w1[:, 0][None, :] + s @ v.T - x * np.sum(v * v, 1)[None, :])
        tb["dw1"].copy_(torch.as_tensor((x.T @ gf[:, None])[:, 0]))
        tb["dv"].copy_(torch.as_tensor(x.T @ (gf[:, None] * s) - ((x * x).T @ gf)[:, None] * v))
        tb["dw0"].copy_(torch.as_tensor([gf.sum()]))
        return torch.as_tensor(dx)

    def scatter_row_grads(self, model, dx, rb):
        so = rb["slot_of"].numpy().reshape(-1).astype(np.int64)
        rows = dx.numpy()[:, model.nd:].reshape(-1, model.k)
        g = rb["gsend"].numpy()
        g[so[so >= 0]] = rows[so >= 0]
        return rb["gsend"]

    def owner_row_sgd(self, model, recv, grecv, lr, tb, rec):
        ids = recv.numpy().astype(np.int64)
        gr = grecv.numpy().astype(np.float64)
        t = model.emb.table_shard.numpy()
        acc = np.zeros(t.shape, np.float64)
        np.add.at(acc, ids[ids >= 0], gr[ids >= 0])
        t[:] = (t.astype(np.float64) - lr * acc).astype(np.float32)

    def deepfm_apply(self, model, tb, lr):
        sh = model.emb
        with torch.no_grad():
            for (L, _), (dW, db) in zip(tb["layers"], tb["dnn_views"]):
                L.kernel -= lr * dW
                L.bias -= lr * db
            sh.w1 -= lr * (tb["dw1"].view(-1, 1) + 2 * model.reg_w * sh.w1)
            sh.v -= lr * (tb["dv"] + 2 * model.reg_v * sh.v)
            sh.w0 -= lr * tb["dw0"]

    # partial protocol (fp64 inside, fp32 buffers like the device path)
    @staticmethod
    def _f32(t):
        return t.view(torch.float32) if t.dtype == torch.int32 else t

    def field_route(self, sh, ids, send, rec=None):
        ids_n = ids.numpy().astype(np.int64)
        B = ids_n.shape[0]
        out = np.full((sh.world, B, sh.slot_stride), -1, np.int64)
        rows = sh.offsets.numpy()[None, :] + ids_n
        for o, (lo, n) in enumerate(sh.owner_field_ranges):
            for j in range(n):
                loc = rows[:, lo + j] - o * sh.rows_per_rank
                m = (loc >= 0) & (loc < sh.rows_per_rank)
                out[o, m, j] = loc[m]
        R = rec or sh.slot_stride
        send.view(-1, R)[:, :sh.slot_stride].copy_(torch.as_tensor(out.reshape(-1, sh.slot_stride), dtype=torch.int32))
        return send

    def owner_partials(self, sh, recv, n_pairs, out, rec=None, poff=0, pst=None):
        lo, n = sh.owner_field_ranges[sh.rank]
        r = recv.numpy().reshape(n_pairs, rec or sh.slot_stride)[:, :sh.slot_stride].astype(np.int64)
        T = sh.table_shard.numpy().astype(np.float64)
        v, w1 = sh.v.numpy().astype(np.float64), sh.w1.numpy().astype(np.float64)[:, 0]
        res = np.zeros((n_pairs, sh.partial_width))
        for j in range(n):
            e = sh.nd + (lo + j) * sh.k + np.arange(sh.k)
            loc = r[:, j]
            x = np.zeros((n_pairs, sh.k))
            x[loc >= 0] = T[loc[loc >= 0]]
            res[:, :sh.kfm] += x @ v[e]
            res[:, sh.kfm] += x @ w1[e]
            res[:, sh.kfm + 1] += (x * x) @ (v[e] ** 2).sum(1)
        P, pst = sh.partial_width, pst or sh.partial_width
        self._f32(out)[poff:].as_strided((n_pairs, P), (pst, 1)).copy_(torch.as_tensor(res, dtype=torch.float32))
        return out

    def combine(self, sh, partials, dense, out, poff=0, pst=None):
        B, nd, kfm = dense.shape[0], sh.nd, sh.kfm
        P, pst = sh.partial_width, pst or sh.partial_width
        flat = self._f32(partials)[poff:]
        p = flat.as_strided((sh.world * B, P), (pst, 1)).numpy().reshape(sh.world, B, P).astype(np.float64).sum(0)
        d = dense.numpy().astype(np.float64)
        v, w1 = sh.v.numpy().astype(np.float64), sh.w1.numpy().astype(np.float64)[:, 0]
        S = p[:, :kfm] + d @ v[:nd]
        lin = p[:, kfm] + d @ w1[:nd]
        q = p[:, kfm + 1] + (d * d) @ (v[:nd] ** 2).sum(1)
        logit = lin + float(sh.w0[0]) + 0.5 * ((S ** 2).sum(1) - q)
        out.copy_(torch.as_tensor(logit.reshape(B, 1), dtype=torch.float32))
        return out

    def pipe(self, sh, recv, send, prev=None, cur=None, nxt=None):
        R = sh.slot_stride + sh.partial_width
        if prev is not None:
            self.combine(sh, recv, prev[0], prev[1], poff=sh.slot_stride, pst=R)
        if cur is not None:
            self.owner_partials(sh, recv, cur.shape[0] * sh.world, send, rec=R, poff=sh.slot_stride, pst=R)
        if nxt is not None:
            self.field_route(sh, nxt[1], send, rec=R)

    # training (fp64 inside)
    def combine_grad(self, sh, partials, dense, labels, scale, logit, gs, loss=None):
        B, nd, kfm, P = dense.shape[0], sh.nd, sh.kfm, sh.partial_width
        p = partials.numpy().reshape(sh.world, B, P).astype(np.float64).sum(0)
        d = dense.numpy().astype(np.float64)
        v, w1 = sh.v.numpy().astype(np.float64), sh.w1.numpy().astype(np.float64)[:, 0]
        S = p[:, :kfm] + d @ v[:nd]
        z = p[:, kfm] + d @ w1[:nd] + float(sh.w0[0]) + 0.5 * ((S ** 2).sum(1) - p[:, kfm + 1] -
                                                                (d * d) @ (v[:nd] ** 2).sum(1))
        t = labels.numpy().astype(np.float64)
        logit.copy_(torch.as_tensor(z.reshape(B, 1), dtype=torch.float32))
        gs[:, :kfm] = torch.as_tensor(S, dtype=torch.float32)
        gs[:, kfm] = torch.as_tensor((1 / (1 + np.exp(-z)) - t) * scale, dtype=torch.float32)
        if loss is not None:
            loss.copy_(torch.as_tensor(np.maximum(z, 0) - z * t + np.log1p(np.exp(-np.abs(z))), dtype=torch.float32))

    def dense_grads(self, sh, dense, gs, grad):
        nd, kfm, d = sh.nd, sh.kfm, sh.d
        x = dense.numpy().astype(np.float64)
        s, g = gs[:, :kfm].numpy().astype(np.float64), gs[:, kfm].numpy().astype(np.float64)
        v = sh.v.numpy().astype(np.float64)
        grad[:nd] = torch.as_tensor(x.T @ g, dtype=torch.float32)
        dv = x.T @ (g[:, None] * s) - ((x * x).T @ g)[:, None] * v[:nd]
        grad[d:d + nd * kfm] = torch.as_tensor(dv.reshape(-1), dtype=torch.float32)
        grad[d * (1 + kfm)] = float(g.sum())

    def owner_grads(self, sh, recv, gs_all, grad, lr, bufs=None):
        lo, n = sh.owner_field_ranges[sh.rank]
        if n == 0:
            return
        k, kfm, d, S = sh.k, sh.kfm, sh.d, sh.slot_stride
        r = recv.numpy().reshape(-1, S)[:, :n].astype(np.int64)
        T = sh.table_shard.numpy().astype(np.float64)
        s, g = gs_all[:, :kfm].numpy().astype(np.float64), gs_all[:, kfm].numpy().astype(np.float64)
        v, w1 = sh.v.numpy().astype(np.float64), sh.w1.numpy().astype(np.float64)[:, 0]
        upd = np.zeros_like(T)
        for j in range(n):
            e = sh.nd + (lo + j) * k + np.arange(k)
            loc = r[:, j]
            x = np.zeros((r.shape[0], k))
            x[loc >= 0] = T[loc[loc >= 0]]
            ve = v[e]
            dx = g[:, None] * (w1[e][None, :] + s @ ve.T - x * (ve * ve).sum(1)[None, :])
            np.add.at(upd, loc[loc >= 0], dx[loc >= 0])
            grad[e] = torch.as_tensor(x.T @ g, dtype=torch.float32)
            dv = x.T @ (g[:, None] * s) - ((x * x).T @ g)[:, None] * ve
            grad[d + e[0] * kfm: d + (e[-1] + 1) * kfm] = torch.as_tensor(dv.reshape(-1), dtype=torch.float32)
        sh.table_shard.copy_(torch.as_tensor(T - lr * upd, dtype=torch.float32))

    def apply(self, sh, grad, lr, reg_w, reg_v):
        d, kfm = sh.d, sh.kfm
        with torch.no_grad():
            sh.w1 -= lr * (grad[:d].reshape(d, 1) + 2 * reg_w * sh.w1)
            sh.v -= lr * (grad[d:d * (1 + kfm)].reshape(d, kfm) + 2 * reg_v * sh.v)
            sh.w0 -= lr * grad[d * (1 + kfm):]

    def bad_flag(self):
        return torch.zeros(1, dtype=torch.int32)

    def clear_flags(self):
        pass


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
        sh.forward_slots(dense0, ids)
        ok_rows = ok_rows and np.array_equal(ops.last_emb.numpy(), expect)
        dense = rng.random((B, 3)).astype(np.float32)
        x = np.concatenate([dense, emb.numpy().reshape(B, -1)], 1)
        fm_sh = O.fm_layer(x, sh.w0.numpy(), sh.w1.numpy(), sh.v.numpy())
        tables = [full[o:o + v] for o, v in zip(sh.offsets.numpy(), vocabs)]
        fm_ref = O.deepfm(None, {"tables": tables, "w0": sh.w0.numpy(), "w1": sh.w1.numpy(), "v": sh.v.numpy(),
                                 "dnn_hidden": [], "dnn_out": (np.zeros((x.shape[1], 1)), np.zeros(1))},
                          nd=3, inputs=(dense, ids.numpy()))[1]
        # partial protocol: owners return FM partials over their fields
        part = sh.forward(torch.as_tensor(dense), ids).numpy()
        rms = float(np.sqrt(np.mean(fm_ref ** 2)))
        ok_part = bool(np.all(np.abs(part - fm_ref) <= 1e-5 * np.maximum(np.abs(fm_ref), rms)))
        # pipelined: 3 batches, one all-to-all each (+1 to drain) == per-batch forward
        d2 = [torch.as_tensor(rng.random((B, 3)).astype(np.float32)) for _ in range(3)]
        i2 = [torch.as_tensor(np.stack([rng.integers(0, v, B) for v in vocabs], 1), dtype=torch.int32)
              for _ in range(2)] + [ids]
        outs = sh.forward_stream(list(zip(d2, i2)))
        for d_, i_, o_ in zip(d2, i2, outs):
            ok_part = ok_part and np.allclose(o_.numpy(), sh.forward(d_, i_).numpy(), rtol=1e-6, atol=1e-7)
        # two-deep (exchange of t+1 beside the pipe of t): the same logits, bit
        # for bit, for every stream length (prologue / drain edge cases)
        for n_ in (1, 2, 3):
            o2 = sh.forward_stream2(list(zip(d2, i2))[:n_])
            ok_part = ok_part and all(torch.equal(a, b) for a, b in zip(o2, outs[:n_] if n_ == 3 else
                                                                       sh.forward_stream(list(zip(d2, i2))[:n_])))
        q.put((rank, ok_rows and ok_part, float(np.max(np.abs(fm_sh - fm_ref))), sh.row_range))
    finally:
        dist.destroy_process_group()


def _train_worker(rank, world, port, vocabs, k, B, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from recommender_system_amd.sharded import ShardedEmbeddingFM
        nd, kfm = 3, 4
        sh = ShardedEmbeddingFM(vocabs, k, nd=nd, kfm=kfm, device="cpu", seed=7, ops=CpuOps())
        with torch.no_grad():
            sh.table_shard.mul_(20.0)  # O(1) activations: a visible update
        shards = [None] * world
        dist.all_gather_object(shards, sh.table_shard.numpy().copy())
        full = np.concatenate(shards).astype(np.float64)
        offs = sh.offsets.numpy()
        p = {"tables": [full[o:o + v] for o, v in zip(offs, vocabs)], "w0": sh.w0.numpy().copy(),
             "w1": sh.w1.numpy().copy(), "v": sh.v.numpy().copy()}
        ok = True
        for step in range(2):
            rngs = [np.random.default_rng(1000 * step + r) for r in range(world)]
            batch = [(rg.random((B, nd)).astype(np.float32),
                      np.stack([rg.integers(0, v, B) for v in vocabs], 1).astype(np.int32),
                      rg.integers(0, 2, B).astype(np.float32)) for rg in rngs]
            dense, ids, t = batch[rank]
            loss = sh.train_step(torch.as_tensor(dense), torch.as_tensor(ids), torch.as_tensor(t), lr=0.5,
                                 reg_w=1e-3, reg_v=2e-3, return_loss=True)
            gd, gi, gt = (np.concatenate([b_[j] for b_ in batch]) for j in range(3))
            p, ce = O.embed_fm_train_step(gd, gi, gt, p, 0.5, 1e-3, 2e-3, nd=nd)
            ok = ok and np.allclose(loss.numpy(), ce[rank * B:(rank + 1) * B], rtol=1e-5, atol=1e-6)
            dist.all_gather_object(shards, sh.table_shard.numpy().copy())
            got = np.concatenate(shards)
            want = np.concatenate(p["tables"])
            ok = ok and np.allclose(got, want, rtol=1e-5, atol=1e-6)
            for name in ("w0", "w1", "v"):
                ok = ok and np.allclose(getattr(sh, name).numpy(), p[name], rtol=1e-5, atol=1e-6)
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


def _deepfm_params(model, full):
    """Oracle parameters of a ShardedDeepFM given the assembled full table
    (copies: the model's tensors change in place when it trains)."""
    c = lambda t: t.detach().cpu().numpy().copy()
    sh = model.emb
    offs = sh.offsets.cpu().numpy()
    return {"tables": [full[o:o + v] for o, v in zip(offs, sh.vocab_sizes)], "w0": c(sh.w0), "w1": c(sh.w1),
            "v": c(sh.v), "dnn_hidden": [(c(l.kernel), c(l.bias)) for l in model.dnn.hidden_layer],
            "dnn_out": (c(model.dnn.output_layer.kernel), c(model.dnn.output_layer.bias))}


def _deepfm_columns(vocabs, nd, k):
    return [[{"feat": f"I{i + 1}"} for i in range(nd)],
            [{"feat": f"C{i + 1}", "feat_onehot_dim": int(v), "embed_dim": k} for i, v in enumerate(vocabs)]]


def _deepfm_worker(rank, world, port, vocabs, k, B, q, dedup=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from recommender_system_amd.sharded import ShardedDeepFM
        nd = 5
        ops = CpuOps()
        m = ShardedDeepFM(_deepfm_columns(vocabs, nd, k), 6, 1e-4, 1e-4, [32, 16], 1, "relu", embed_dim=k,
                          device="cpu", seed=3, ops=ops, dedup=dedup)
        with torch.no_grad():
            m.table_shard.mul_(20.0)  # O(1) embeddings: the DNN sees them
        shards = [None] * world
        dist.all_gather_object(shards, m.table_shard.numpy().copy())
        full = np.concatenate(shards)
        p = _deepfm_params(m, full)
        # replicated parameters are identical on every rank
        ws = [None] * world
        dist.all_gather_object(ws, {n: t.detach().numpy().copy() for n, t in m.keras_weights().items()})
        ok = all(np.array_equal(ws[0][n], ws[r][n]) for r in range(world) for n in ws[0])
        rng = np.random.default_rng(300 + rank)
        for step in range(2):
            dense = rng.random((B, nd)).astype(np.float32)
            ids = np.stack([rng.integers(0, v, B) for v in vocabs], 1).astype(np.int32)
            if step == 1:
                ids[0, 3] = vocabs[3] - 1  # last row of a field
            y = m.forward((torch.as_tensor(dense), torch.as_tensor(ids))).numpy()
            ref, _, _ = O.deepfm(None, p, nd=nd, inputs=(dense, ids))
            rows = m.emb.offsets.numpy()[None, :] + ids
            ok = ok and np.array_equal(ops.last_emb, full[rows.reshape(-1)].astype(np.float64))
            ok = ok and bool(np.all(np.abs(y - ref) <= 1e-5 * np.abs(ref)))
        # the pipelined stream (batch t+1's exchange beside batch t's forward,
        # two buffer slots) gives every batch the per-batch forward's output
        batches = [(torch.as_tensor(rng.random((B, nd)).astype(np.float32)),
                    torch.as_tensor(np.stack([rng.integers(0, v, B) for v in vocabs], 1).astype(np.int32)))
                   for _ in range(3)]
        outs = m.forward_stream(batches)
        for (d_, i_), o_ in zip(batches, outs):
            ok = ok and np.array_equal(o_.numpy(), m.forward((d_, i_)).numpy())
        q.put((rank, bool(ok), m.emb.owner_field_ranges))
    finally:
        dist.destroy_process_group()


def _global_masks(seed, world, offset, B, widths, rate):
    """Dropout multipliers of the global batch: every rank's own draws
    (sharded.dropout_seed), stacked in rank order."""
    from recommender_system_amd.sharded import dropout_seed
    from tests.helpers import dropout_masks
    per = [dropout_masks(dropout_seed(seed, r), offset, B, widths, rate)[0] for r in range(world)]
    return [np.concatenate([per[r][i] for r in range(world)]) for i in range(len(widths))]


def _deepfm_train_worker(rank, world, port, vocabs, k, B, q, dedup=None, drop=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from recommender_system_amd.sharded import ShardedDeepFM
        nd, lr = 5, 0.5
        m = ShardedDeepFM(_deepfm_columns(vocabs, nd, k), 6, 1e-3, 2e-3, [32, 16], 1, "relu", embed_dim=k,
                          device="cpu", seed=3, ops=CpuOps(), dedup=dedup)
        if dedup is not None and dedup < 0.05:
            m._dedup_cap = lambda B_: 1  # every step overflows: the collective fallback must stay exact
        with torch.no_grad():
            m.table_shard.mul_(20.0)  # O(1) embeddings: visible row updates
        shards = [None] * world
        dist.all_gather_object(shards, m.table_shard.numpy().copy())
        p = _deepfm_params(m, np.concatenate(shards).astype(np.float64))
        ok = True
        for step in range(2):
            rngs = [np.random.default_rng(500 * step + r) for r in range(world)]
            batch = [(rg.random((B, nd)).astype(np.float32),
                      np.stack([rg.integers(0, v, B) for v in vocabs], 1).astype(np.int32),
                      rg.integers(0, 2, B).astype(np.float32)) for rg in rngs]
            for b_ in batch:
                b_[1][:3, 1] = 0  # repeated rows inside and across ranks
            dense, ids, t = batch[rank]
            off = m._dropout().offset
            loss = m.train_step((torch.as_tensor(dense), torch.as_tensor(ids)), torch.as_tensor(t), lr=lr,
                                return_loss=True, dropout=None if drop else False)
            gd, gi, gt = (np.concatenate([b_[j] for b_ in batch]) for j in range(3))
            masks = _global_masks(3, world, off, B, [32, 16], 0.2) if drop else None
            p, ce = O.deepfm_train_step(gd, gi, gt, p, lr, 1e-3, 2e-3, nd=nd, masks=masks)
            ok = ok and np.allclose(loss.numpy(), ce[rank * B:(rank + 1) * B], rtol=1e-5, atol=1e-6)
            dist.all_gather_object(shards, m.table_shard.numpy().copy())
            ok = ok and np.allclose(np.concatenate(shards), np.concatenate(p["tables"]), rtol=1e-5, atol=1e-6)
            mine = _deepfm_params(m, np.concatenate(shards))
            for n in ("w0", "w1", "v"):
                ok = ok and np.allclose(mine[n], p[n], rtol=1e-5, atol=1e-6)
            for (W1, b1), (W2, b2) in zip(mine["dnn_hidden"] + [mine["dnn_out"]], p["dnn_hidden"] + [p["dnn_out"]]):
                ok = ok and np.allclose(W1, W2, rtol=1e-5, atol=1e-6) and np.allclose(b1, b2, rtol=1e-5, atol=1e-6)
        if dedup is not None and dedup < 0.05:
            ok = ok and m.ops.fallbacks == 2  # both steps fell back
        q.put((rank, bool(ok)))
    except Exception as e:  # report instead of leaving the parent waiting on the queue
        q.put((rank, f"{type(e).__name__}: {e}"))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,dedup,drop", [(2, None, True), (3, None, False), (2, 1.0, False), (3, 0.01, True)])
def test_sharded_deepfm_train_step_gloo(world, dedup, drop):
    """ShardedDeepFM.train_step over gloo (world 2, 3): forward row exchange,
    each rank's local DeepFM backward scaled to the global batch, the REVERSE
    all-to-all of dL/drow to the owners (row-sparse SGD of each shard,
    duplicates across ranks summed), the all-reduce of the flat replicated
    gradient — every shard, w0 / w1 / v and every DNN layer equal
    O.deepfm_train_step on the concatenated global batch, over 2 steps.
    dedup: the distinct-row exchange (each owner gets every distinct row
    once per rank, row gradients summed at the requester); 0.01 = a tiny
    capacity that overflows, so every step falls back (collectively) to
    the field-range records and must still be exact.  drop: DNNLayer's
    Dropout(0.2) in training mode, each rank drawing its own masks (the
    oracle gets the same multipliers, stacked in rank order)."""
    vocabs = [50, 7, 300, 1, 120, 33]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_deepfm_train_worker, args=(r, world, port, vocabs, 4, 19, q, dedup, drop))
             for r in range(world)]
    for p_ in procs:
        p_.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p_ in procs:
        p_.join(timeout=60)
        assert p_.exitcode == 0
    for rank, ok in res:
        assert ok is True, f"rank {rank}: sharded DeepFM training step differs from the oracle ({ok})"


@pytest.mark.parametrize("world,dedup", [(2, None), (3, None), (3, 1.0)])
def test_sharded_deepfm_gloo(world, dedup):
    """ShardedDeepFM over gloo (world 2, 3; config 5's protocol): row route ->
    all-to-all of row ids -> owner gather -> all-to-all of rows -> DeepFM from
    the exchange buffer.  Every lookup gets exactly its row of the global table
    (fields straddle owners: the vocabularies are uneven) and the output
    equals O.deepfm on the unsharded model at 1e-5 relative (post-sigmoid)."""
    rng = np.random.default_rng(world + 11)
    vocabs = [int(v) for v in rng.integers(1, 400, 9)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_deepfm_worker, args=(r, world, port, vocabs, 4, 37, q, dedup)) for r in range(world)]
    for p_ in procs:
        p_.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p_ in procs:
        p_.join(timeout=60)
    assert all(ok for _, ok, _ in res), res


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_train_step_gloo(world):
    """ShardedEmbeddingFM.train_step over gloo (world 2, 3): forward partials,
    the [s | g] all-gather, owner row gradients + row SGD, the parameter
    all-reduce — every rank's shard and the replicated w0 / w1 / v equal the
    oracle's SGD step on the concatenated global batch, over 2 steps."""
    vocabs = [50, 7, 300, 1, 120]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_train_worker, args=(r, world, port, vocabs, 4, 17, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok in res:
        assert ok, f"rank {rank}: sharded training step differs from the oracle"


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
    a = sh.forward_slots(dense, ids)           # fixed-capacity row slots
    e = sh.forward_exact(dense, ids)           # counts + variable splits
    pp = sh.forward(dense, ids)                # owner FM partials (default)
    ids2 = torch.as_tensor(np.stack([rng.integers(0, v, B) for v in vocabs], 1), dtype=torch.int32, device=gpu)
    dense2 = torch.rand(B, 13, device=gpu)
    st = sh.forward_stream([(dense, ids), (dense2, ids2), (dense, ids)])  # pipelined, one launch per step
    np.testing.assert_allclose(st[1].cpu().numpy(), sh.forward(dense2, ids2).cpu().numpy(), rtol=1e-6, atol=1e-7)
    sh._slot_bufs = None
    sh.capacity = lambda n: 7                  # forced overflow -> exact fallback
    f = sh.forward_slots(dense, ids)
    b = torch.empty(B, 1, device=gpu)
    _lib.call("rs_embed_fm_fwd", ids.data_ptr(), 0, 26, dense.data_ptr(), 13, 13, sh.table_shard.data_ptr(),
              sh.offsets.data_ptr(), sh.vocab.data_ptr(), 26, 16, sh.prepared.data_ptr(), sh.w0.data_ptr(), 10,
              b.data_ptr(), None, B, None, _lib.stream())
    np.testing.assert_allclose(a.cpu().numpy(), b.cpu().numpy(), rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(e.cpu().numpy(), b.cpu().numpy(), rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(f.cpu().numpy(), b.cpu().numpy(), rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(pp.cpu().numpy(), b.cpu().numpy(), rtol=1e-6, atol=1e-6)
    for o in (st[0], st[2]):
        np.testing.assert_allclose(o.cpu().numpy(), b.cpu().numpy(), rtol=1e-6, atol=1e-6)
    bad = ids.clone()
    bad[3, 5] = vocabs[5]
    sh.capacity = lambda n: max(n, 1)
    sh._slot_bufs = None
    with pytest.raises(IndexError):
        sh.forward_slots(dense, bad)
    with pytest.raises(IndexError):
        sh.forward(dense, bad)


@pytest.mark.gpu
@pytest.mark.parametrize("fused", [False, True])
@pytest.mark.parametrize("world,k,kfm", [(8, 16, 10), (3, 16, 10), (2, 8, 20), (5, 4, 3)])
def test_gpu_partial_protocol_simulated_world(gpu, world, k, kfm, fused):
    """The partial protocol's three kernels at world > 1 in ONE process: each
    simulated rank routes its own batch, the all-to-all is done as a block
    transpose, every owner runs rs_shard_owner_fm on its shard, and every
    requester's rs_shard_fm_combine must equal the unsharded fused kernel
    (rs_embed_fm_fwd over the concatenated table) and the fp64 oracle.
    fused: the pipelined layout (row ids and partials interleaved in one
    record per peer and sample, as forward_stream exchanges them)."""
    from recommender_system_amd import _lib
    from recommender_system_amd.sharded import ShardedEmbeddingFM
    rng = np.random.default_rng(world * 100 + k)
    vocabs = [int(v) for v in rng.integers(1, 4000, 26)]
    vocabs[7] = 20000  # one field straddles several owners
    B, nd = 257, 13
    shs = [ShardedEmbeddingFM(vocabs, k, nd, kfm, device=gpu, seed=11, table_init=False, world=world, rank=r)
           for r in range(world)]
    full = torch.empty(shs[0].total_rows, k, device=gpu).uniform_(-0.05, 0.05)
    for sh in shs:
        lo, hi = sh.row_range
        sh.table_shard = full[lo:hi].contiguous()
    ids = [torch.as_tensor(np.stack([rng.integers(0, v, B) for v in vocabs], 1), dtype=torch.int32, device=gpu)
           for _ in range(world)]
    dense = [torch.rand(B, nd, device=gpu) for _ in range(world)]
    S, P = shs[0].slot_stride, shs[0].partial_width
    R = S + P if fused else S          # words per row-id record
    poff, pst = (S, S + P) if fused else (0, P)
    sends = [sh.ops.field_route(sh, ids[r], torch.full((world * B * R,), 7, dtype=torch.int32, device=gpu), rec=R)
             for r, sh in enumerate(shs)]
    id_words = [x.view(world * B, R)[:, :S].clone() for x in sends]
    if fused:  # the route left the partial words alone
        assert all(bool((x.view(world * B, R)[:, S:] == 7).all()) for x in sends)
    # all-to-all #1: owner o receives block o of every requester, requester-major
    recvs = [torch.cat([sends[r].view(world, B * R)[o] for r in range(world)]) for o in range(world)]
    pouts = [sh.ops.owner_partials(sh, recvs[o], world * B, sends[o] if fused else
                                   torch.empty(world * B * P, device=gpu), rec=R, poff=poff, pst=pst)
             for o, sh in enumerate(shs)]
    if fused:  # the owner wrote only the partial words: row-id words intact
        for o in range(world):
            assert torch.equal(pouts[o].view(world * B, R)[:, :S], id_words[o])
    # all-to-all #2: requester r receives block r of every owner, owner-major
    blk = B * (R if fused else P)
    pins = [torch.cat([pouts[o].view(world, blk)[r] for o in range(world)]) for r in range(world)]
    for r, sh in enumerate(shs):
        got = sh.ops.combine(sh, pins[r], dense[r], torch.empty(B, 1, device=gpu), poff=poff, pst=pst)
        ref = torch.empty(B, 1, device=gpu)
        _lib.call("rs_embed_fm_fwd", ids[r].data_ptr(), 0, 26, dense[r].data_ptr(), nd, nd, full.data_ptr(),
                  sh.offsets.data_ptr(), sh.vocab.data_ptr(), 26, k, sh.prepared.data_ptr(), sh.w0.data_ptr(), kfm,
                  ref.data_ptr(), None, B, None, _lib.stream())
        g, f = got.cpu().numpy(), ref.cpu().numpy()
        rms = float(np.sqrt(np.mean(f ** 2)))
        assert np.all(np.abs(g - f) <= 1e-5 * np.maximum(np.abs(f), rms)), (r, float(np.max(np.abs(g - f))))
        T = full.cpu().numpy().astype(np.float64)
        offs = sh.offsets.cpu().numpy()
        tables = [T[o:o + v] for o, v in zip(offs, vocabs)]
        oracle = O.deepfm(None, {"tables": tables, "w0": sh.w0.cpu().numpy(), "w1": sh.w1.cpu().numpy(),
                                 "v": sh.v.cpu().numpy(), "dnn_hidden": [],
                                 "dnn_out": (np.zeros((nd + 26 * k, 1)), np.zeros(1))},
                          nd=nd, inputs=(dense[r].cpu().numpy(), ids[r].cpu().numpy()))[1]
        rms = float(np.sqrt(np.mean(oracle ** 2)))
        assert np.all(np.abs(g - oracle) <= 1e-5 * np.maximum(np.abs(oracle), rms))
    for sh in shs:
        sh.ops.check()


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


@pytest.mark.gpu
def test_gpu_slot_bucketize_workspace_reuse(gpu):
    """One HipShardOps (one workspace) across calls whose lookup count shrinks
    (B 4096 -> 32, a short last batch) and after the exact protocol filled the
    shared hist region: the single-pass scan's control word lives at a fixed
    offset, so every call still equals the numpy slot double."""
    from recommender_system_amd.sharded import HipShardOps
    rng = np.random.default_rng(77)
    vocabs = rng.integers(1, 5000, 26)
    offs = np.concatenate([[0], np.cumsum(vocabs)[:-1]])
    world = 8
    rpr = int(np.ceil(vocabs.sum() / world))
    ops = HipShardOps(gpu)
    t = lambda a, dt=None: torch.as_tensor(a, dtype=dt, device=gpu)
    for step, B in enumerate([4096, 32, "exact", 32, 4096, 7]):
        if B == "exact":
            ids = np.stack([rng.integers(0, v, 2048) for v in vocabs], 1)
            c, _, _ = ops.bucketize(t(ids, torch.int32), t(offs), t(vocabs), rpr, world)
            rc, _, _ = CpuOps().bucketize(torch.as_tensor(ids), torch.as_tensor(offs), None, rpr, world)
            np.testing.assert_array_equal(c.cpu().numpy(), rc.numpy())
            continue
        n = B * 26
        cap = min(n, int(np.ceil(1.15 * n / world)) + 64)
        bufs = {"counts": torch.empty(world, dtype=torch.int32, device=gpu),
                "slot_of": torch.empty(n, dtype=torch.int32, device=gpu),
                "send": torch.full((world * cap,), -1, dtype=torch.int32, device=gpu),
                "overflow": torch.zeros(1, dtype=torch.int32, device=gpu)}
        ids = np.stack([rng.integers(0, v, B) for v in vocabs], 1)
        so, send = ops.slot_bucketize(t(ids, torch.int32), t(offs), t(vocabs), rpr, world, cap, bufs)
        ref = CpuOps()
        rso, rsend = ref.slot_bucketize(torch.as_tensor(ids), torch.as_tensor(offs), None, rpr, world, cap)
        np.testing.assert_array_equal(so.cpu().numpy(), rso.numpy(), err_msg=f"call {step} (B={B})")
        np.testing.assert_array_equal(send.cpu().numpy(), rsend.numpy(), err_msg=f"call {step} (B={B})")
        assert bool(bufs["overflow"].item()) == ref.overflow


@pytest.mark.gpu
@pytest.mark.parametrize("world", [1, 2, 8])
def test_gpu_pipe_kernel_simulated_world(gpu, world):
    """rs_shard_fm_pipe (combine t-1 | owner t | route t+1 in one launch) over
    a stream of 3 batches per simulated rank, the all-to-all done as a block
    transpose of the fused records: every batch's logit equals the unsharded
    fused kernel."""
    from recommender_system_amd import _lib
    from recommender_system_amd.sharded import ShardedEmbeddingFM
    rng = np.random.default_rng(world + 40)
    vocabs = [int(v) for v in rng.integers(1, 3000, 26)]
    B, nd, k, kfm, T = 300, 13, 16, 10, 3
    shs = [ShardedEmbeddingFM(vocabs, k, nd, kfm, device=gpu, seed=5, table_init=False, world=world, rank=r)
           for r in range(world)]
    full = torch.empty(shs[0].total_rows, k, device=gpu).uniform_(-0.05, 0.05)
    for sh in shs:
        lo, hi = sh.row_range
        sh.table_shard = full[lo:hi].contiguous()
    batches = [[(torch.rand(B, nd, device=gpu),
                 torch.as_tensor(np.stack([rng.integers(0, v, B) for v in vocabs], 1), dtype=torch.int32,
                                 device=gpu)) for _ in range(T)] for _ in range(world)]
    outs = [[torch.full((B, 1), float("nan"), device=gpu) for _ in range(T)] for _ in range(world)]
    for r, sh in enumerate(shs):
        sh.pipe_route(batches[r][0][1])
    R = shs[0].slot_stride + shs[0].partial_width
    for t in range(T + 1):
        sends = [sh._sbufs(B)["send"] for sh in shs]
        recvs = [torch.cat([sends[q].view(world, B * R)[o] for q in range(world)]) for o in range(world)]
        for r, sh in enumerate(shs):
            prev = (batches[r][t - 1][0], outs[r][t - 1]) if t > 0 else None
            cur = batches[r][t][1] if t < T else None
            nxt = batches[r][t + 1] if t + 1 < T else None
            sh.ops.pipe(sh, recvs[r], sends[r], prev=prev, cur=cur, nxt=nxt)
    for r, sh in enumerate(shs):
        for t in range(T):
            dense, ids = batches[r][t]
            ref = torch.empty(B, 1, device=gpu)
            _lib.call("rs_embed_fm_fwd", ids.data_ptr(), 0, 26, dense.data_ptr(), nd, nd, full.data_ptr(),
                      sh.offsets.data_ptr(), sh.vocab.data_ptr(), 26, k, sh.prepared.data_ptr(), sh.w0.data_ptr(),
                      kfm, ref.data_ptr(), None, B, None, _lib.stream())
            g, f = outs[r][t].cpu().numpy(), ref.cpu().numpy()
            rms = float(np.sqrt(np.mean(f ** 2)))
            assert np.all(np.abs(g - f) <= 1e-5 * np.maximum(np.abs(f), rms)), (r, t)
        sh.ops.check()


@pytest.mark.gpu
@pytest.mark.parametrize("world,k,kfm", [(1, 16, 10), (3, 16, 10), (8, 16, 10), (5, 4, 3)])
def test_gpu_sharded_train_step_simulated_world(gpu, world, k, kfm):
    """The sharded training step's HIP kernels (rs_shard_fm_combine_grad,
    rs_fm_param_grads_strided, rs_shard_owner_fm_grad, rs_embedding_sgd on the
    received records, rs_sgd_update) at world 1 (ShardedEmbeddingFM.train_step
    itself) and simulated worlds 3 / 5 / 8 in one process (all-to-all = block
    transpose, all-gather = concatenation, all-reduce = sum in rank order),
    2 steps: every rank's shard and the replicated parameters equal the fp64
    oracle's SGD step on the concatenated global batch."""
    from tests.helpers import assert_scaled_close
    from recommender_system_amd.sharded import ShardedEmbeddingFM
    rng = np.random.default_rng(world * 31 + k)
    vocabs = [int(v) for v in rng.integers(1, 60, 26)]
    vocabs[7] = 900  # one field straddles several owners; many repeated rows elsewhere
    B, nd = 129, 13
    shs = [ShardedEmbeddingFM(vocabs, k, nd, kfm, device=gpu, seed=11, table_init=False, world=world, rank=r)
           for r in range(world)]
    full = torch.empty(shs[0].total_rows, k, device=gpu).uniform_(-1.0, 1.0)
    for sh in shs:
        lo, hi = sh.row_range
        sh.table_shard = full[lo:hi].contiguous()
    offs = shs[0].offsets.cpu().numpy()
    T = full.cpu().numpy().astype(np.float64)
    p = {"tables": [T[o:o + v] for o, v in zip(offs, vocabs)], "w0": shs[0].w0.cpu().numpy(),
         "w1": shs[0].w1.cpu().numpy(), "v": shs[0].v.cpu().numpy()}
    lr, rw, rv = 0.5, 1e-3, 2e-3
    for step in range(2):
        dense = [torch.as_tensor(rng.random((B, nd)), dtype=torch.float32, device=gpu) for _ in range(world)]
        ids = [torch.as_tensor(np.stack([rng.integers(0, v, B) for v in vocabs], 1), dtype=torch.int32, device=gpu)
               for _ in range(world)]
        lab = [torch.as_tensor(rng.integers(0, 2, B), dtype=torch.float32, device=gpu) for _ in range(world)]
        if world == 1:
            losses = [shs[0].train_step(dense[0], ids[0], lab[0], lr=lr, reg_w=rw, reg_v=rv, return_loss=True)]
        else:
            S, P = shs[0].slot_stride, shs[0].partial_width
            pbs = [sh._pbufs(B) for sh in shs]
            tbs = [sh._tbufs(B) for sh in shs]
            sends = [sh.ops.field_route(sh, ids[r], pbs[r]["send"]) for r, sh in enumerate(shs)]
            recvs = [torch.cat([sends[r].view(world, B * S)[o] for r in range(world)]) for o in range(world)]
            pouts = [sh.ops.owner_partials(sh, recvs[o], world * B, pbs[o]["pout"]) for o, sh in enumerate(shs)]
            pins = [torch.cat([pouts[o].view(world, B * P)[r] for o in range(world)]) for r in range(world)]
            losses = []
            for r, sh in enumerate(shs):
                losses.append(torch.empty(B, device=gpu))
                sh.ops.combine_grad(sh, pins[r], dense[r], lab[r], 1.0 / (world * B), tbs[r]["logit"], tbs[r]["gs"],
                                    losses[-1])
            gs_all = torch.cat([tb["gs"] for tb in tbs])
            for r, sh in enumerate(shs):
                tbs[r]["grad"].zero_()
                sh.ops.dense_grads(sh, dense[r], tbs[r]["gs"], tbs[r]["grad"])
                sh.ops.owner_grads(sh, recvs[r], gs_all, tbs[r]["grad"], lr, tbs[r])
            total = tbs[0]["grad"].clone()
            for tb in tbs[1:]:
                total += tb["grad"]
            for sh in shs:
                sh.ops.apply(sh, total, lr, rw, rv)
        cat = lambda xs: np.concatenate([x.cpu().numpy() for x in xs])
        p, ce = O.embed_fm_train_step(cat(dense), cat(ids), cat(lab), p, lr, rw, rv, nd=nd)
        assert_scaled_close(cat(losses), ce, what=f"step {step} loss")
        got = np.concatenate([sh.table_shard.cpu().numpy() for sh in shs])
        assert_scaled_close(got, np.concatenate(p["tables"]), what=f"step {step} table")
        for sh in shs:
            for name in ("w1", "v"):
                assert_scaled_close(getattr(sh, name), p[name], what=f"step {step} {name}")
            # w0 = -lr * sum_b g_b per step, a signed sum of the global batch
            # (|g_b| <= 1/(world*B)): its fp32 error scales with lr * sum|g|
            # <= lr per step, not with |w0| (which cancels toward 0)
            w0, r0 = float(sh.w0.cpu()[0]), float(np.asarray(p["w0"]).reshape(-1)[0])
            assert abs(w0 - r0) <= 1e-5 * max(abs(r0), lr * (step + 1)), (step, w0, r0)
    for sh in shs:
        sh.ops.check()


def _compact_deepfm_reference(models, dense, ids):
    """O.deepfm for a batch of global ids without assembling the global table
    on the host: per field, only the touched rows (read from their owners'
    shards) and ids remapped into them."""
    m0 = models[0]
    sh0 = m0.emb
    offs, rpr = sh0.offsets.cpu().numpy(), sh0.rows_per_rank
    tables, rid = [], np.empty_like(ids)
    for c in range(ids.shape[1]):
        u, inv = np.unique(ids[:, c], return_inverse=True)
        rows = offs[c] + u
        own = np.minimum(rows // rpr, len(models) - 1)
        t = np.empty((u.size, sh0.k), np.float32)
        for o in np.unique(own):
            sel = own == o
            loc = torch.as_tensor(rows[sel] - o * rpr, device=models[o].table_shard.device)
            t[sel] = models[o].table_shard[loc].cpu().numpy()
        tables.append(t)
        rid[:, c] = inv
    c_ = lambda t: t.detach().cpu().numpy()
    p = {"tables": tables, "w0": c_(sh0.w0), "w1": c_(sh0.w1), "v": c_(sh0.v),
         "dnn_hidden": [(c_(l.kernel), c_(l.bias)) for l in m0.dnn.hidden_layer],
         "dnn_out": (c_(m0.dnn.output_layer.kernel), c_(m0.dnn.output_layer.bias))}
    return O.deepfm(None, p, nd=m0.nd, inputs=(dense, rid))[0]


def _simulated_deepfm_step(models, batches):
    """One ShardedDeepFM forward of every rank of a simulated world on one
    GPU: each rank's row route, the all-to-alls as block transposes of the
    records, every owner's gather, every requester's fused DeepFM."""
    W = len(models)
    B = batches[0][1].shape[0]
    k = models[0].k
    rbs = [m._rbufs(B) for m in models]
    for m, rb, (_, ids) in zip(models, rbs, batches):
        m.route(ids, rb)
    for o in range(W):
        rbs[o]["recv"].view(W, -1).copy_(torch.stack([rbs[r]["send"].view(W, -1)[o] for r in range(W)]))
    for m, rb in zip(models, rbs):
        m.serve(rb["recv"], rb["reply"])
    for r in range(W):
        rbs[r]["got"].view(W, -1, k).copy_(torch.stack([rbs[o]["reply"].view(W, -1, k)[r] for o in range(W)]))
    outs = []
    for m, rb, (dense, _) in zip(models, rbs, batches):
        outs.append(m.finish(dense, rb["got"], rb, torch.empty(B, 1, device=dense.device)))
    return outs


@pytest.mark.gpu
@pytest.mark.parametrize("world,vocab,B,k", [(2, None, 300, 16), (3, None, 257, 8), (8, None, 256, 16),
                                             (8, 3846154, 512, 16)])
def test_gpu_sharded_deepfm_simulated_world(gpu, world, vocab, B, k):
    """ShardedDeepFM (config 5) on simulated worlds of 2 / 3 / 8 ranks on one
    GPU — rs_shard_row_route, the all-to-alls as block transposes,
    rs_gather_rows at every owner, rs_deepfm_fwd from the exchange buffer —
    equals O.deepfm on the unsharded model at 1e-5 relative (post-sigmoid).
    The last case is config 5's table: 26 fields x 3,846,154 rows = 1e8 rows
    (6.4 GB) over 8 owners, 4 fields per owner, straddling fields."""
    from recommender_system_amd.sharded import ShardedDeepFM
    from tests.helpers import assert_rel_close
    rng = np.random.default_rng(world * 7 + k)
    vocabs = [int(vocab)] * 26 if vocab else [int(v) for v in rng.integers(1, 5000, 26)]
    nd, kfm = 13, 10
    cols = _deepfm_columns(vocabs, nd, k)
    models = [ShardedDeepFM(cols, kfm, 1e-4, 1e-4, [256, 128, 64], 1, "relu", embed_dim=k, device=gpu, seed=5,
                            world=world, rank=r) for r in range(world)]
    for m in models:
        with torch.no_grad():
            m.table_shard.mul_(10.0)  # O(0.5) embeddings: the tower and the FM both matter
    batches = []
    for r in range(world):
        ids = np.stack([rng.integers(0, v, B) for v in vocabs], 1).astype(np.int32)
        ids[0] = np.array(vocabs) - 1  # last row of every field
        batches.append((torch.rand(B, nd, device=gpu), torch.as_tensor(ids, device=gpu)))
    outs = _simulated_deepfm_step(models, batches)
    for r in range(world):
        ref = _compact_deepfm_reference(models, batches[r][0].cpu().numpy(), batches[r][1].cpu().numpy())
        assert_rel_close(outs[r], ref, what=f"rank {r}")
    for m in models:
        assert int(m.ops.err.item()) == 0


@pytest.mark.gpu
def test_gpu_sharded_deepfm_world1(gpu):
    """World 1: the direct path (rs_deepfm_fwd on the shard = whole table) and
    the row protocol (route -> serve -> DeepFM from the exchange buffer, the
    exchange being the identity) both equal O.deepfm; an out-of-range id
    raises IndexError on both paths; int64 and packed-float inputs work."""
    from recommender_system_amd.sharded import ShardedDeepFM
    from tests.helpers import assert_rel_close
    rng = np.random.default_rng(1)
    vocabs = [1000, 50, 3000, 7] * 6 + [11, 12]
    cols = _deepfm_columns(vocabs, 13, 16)
    m = ShardedDeepFM(cols, 10, 1e-4, 1e-4, [256, 128, 64], 1, "relu", embed_dim=16, device=gpu, seed=2)
    B = 300
    ids = np.stack([rng.integers(0, v, B) for v in vocabs], 1)
    dense = rng.random((B, 13)).astype(np.float32)
    ref = _compact_deepfm_reference([m], dense, ids)
    direct = m.forward((dense, ids.astype(np.int64)))
    assert_rel_close(direct, ref, what="direct")
    X = np.concatenate([dense, ids], 1)  # the reference's packed X
    assert_rel_close(m.forward(X), ref, what="packed X")
    m.force_rows = True
    rows = m.forward((dense, ids.astype(np.int32)))
    assert_rel_close(rows, ref, what="row protocol")
    bad = ids.copy()
    bad[5, 3] = vocabs[3]
    for force in (False, True):
        m.force_rows = force
        with pytest.raises(IndexError):
            m.forward((dense, bad))


@pytest.mark.gpu
def test_gpu_rccl_self_exchange(gpu):
    """The sharded paths with their RCCL all-to-alls forced on (a 1-rank nccl
    group, eager and HIP-graph captured) equal the same paths without the
    exchange, bit for bit (tests/rccl_selfcheck.py, in a child process with
    its own time limit)."""
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, os.path.join(here, "rccl_selfcheck.py")], capture_output=True, text=True,
                       timeout=100)
    assert r.returncode == 0 and "RCCL OK" in r.stdout, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])


def _simulated_deepfm_train(models, batches, labels, lr, rate=0.0):
    """One ShardedDeepFM.train_step of every rank of a simulated world on one
    GPU, step by step: the forward row exchange (block transposes), every
    rank's deepfm_grads + rs_scatter_rows, the reverse all-to-all of the row
    gradients (block transpose), every owner's row SGD, the all-reduce of the
    flat replicated gradient (sum in rank order), every rank's SGD."""
    W = len(models)
    B = batches[0][1].shape[0]
    k = models[0].k
    rbs = [m._rbufs(B) for m in models]
    tbs = [m._tbufs(B) for m in models]
    for m, rb, (_, ids) in zip(models, rbs, batches):
        m.route(ids, rb)
        if rb["dedup"]:  # this helper has no fallback: the capacity must hold
            assert not bool(m.ops.overflow_flag(rb).item())
    for o in range(W):
        rbs[o]["recv"].view(W, -1).copy_(torch.stack([rbs[r]["send"].view(W, -1)[o] for r in range(W)]))
    for m, rb in zip(models, rbs):
        m.serve(rb["recv"], rb["reply"])
    for r in range(W):
        rbs[r]["got"].view(W, -1, k).copy_(torch.stack([rbs[o]["reply"].view(W, -1, k)[r] for o in range(W)]))
    losses = []
    for m, rb, tb, (dense, _), t in zip(models, rbs, tbs, batches, labels):
        losses.append(torch.empty(B, device=dense.device))
        dx = m.ops.deepfm_grads(m, rb["got"], rb, dense, t, 1.0 / (W * B), tb, losses[-1], drop=m._draws(B, rate))
        if rb["dedup"]:
            m.ops.dedup_grads(m, dx, rb)
        else:
            m.ops.scatter_row_grads(m, dx, rb)
    for o in range(W):
        rbs[o]["grecv"].view(W, -1, k).copy_(torch.stack([rbs[r]["gsend"].view(W, -1, k)[o] for r in range(W)]))
    for m, rb, tb in zip(models, rbs, tbs):
        m.ops.owner_row_sgd(m, rb["recv"], rb["grecv"], lr, tb, rb["rec"])
    total = tbs[0]["flat"].clone()
    for tb in tbs[1:]:
        total += tb["flat"]
    for m, tb in zip(models, tbs):
        tb["flat"].copy_(total)
        m.ops.deepfm_apply(m, tb, lr)
    return losses


@pytest.mark.gpu
@pytest.mark.parametrize("world,B,k,dedup,drop", [(1, 300, 16, None, True), (2, 200, 16, None, False),
                                                  (3, 129, 8, None, True), (8, 128, 16, None, True),
                                                  (1, 300, 16, 1.0, False), (3, 129, 8, 1.0, False),
                                                  (8, 128, 16, 1.0, True)])
def test_gpu_sharded_deepfm_train_simulated_world(gpu, world, B, k, dedup, drop):
    """ShardedDeepFM.train_step's HIP path (rs_embed_gather from the exchange
    buffer, rs_dense_fwd / rs_fm_fwd with saved activations,
    rs_head_grad_scaled, the rs_gemm DNN backward, rs_fm_x_grad /
    rs_fm_param_grads, rs_scatter_rows into the slot layout, the reverse
    all-to-all, the owners' rs_embedding_sgd on the ids they served, the
    flat-gradient all-reduce, rs_sgd_update) at world 1 (train_step itself)
    and simulated worlds 2 / 3 / 8, 2 steps with rows repeated within and
    across ranks: every shard, w0 / w1 / v and every DNN layer equal
    O.deepfm_train_step on the concatenated global batch.  dedup: the
    distinct-row exchange (rs_shard_dedup_route / rs_shard_dedup_grad).
    drop: DNNLayer's Dropout(0.2) in training, each rank's own rs_dropout
    draws (the oracle gets the same multipliers)."""
    from recommender_system_amd.sharded import ShardedDeepFM
    from tests.helpers import assert_scaled_close
    rng = np.random.default_rng(world * 13 + k)
    vocabs = [int(v) for v in rng.integers(1, 400, 26)]
    vocabs[5] = 3000  # straddles owners
    nd, kfm, lr, rw, rv = 13, 10, 0.5, 1e-3, 2e-3
    cols = _deepfm_columns(vocabs, nd, k)
    models = [ShardedDeepFM(cols, kfm, rw, rv, [64, 32], 1, "relu", embed_dim=k, device=gpu, seed=9,
                            world=world, rank=r, dedup=dedup) for r in range(world)]
    for m in models:
        with torch.no_grad():
            m.table_shard.mul_(10.0)  # O(1) embeddings: visible row updates
            for l in m.dnn._layers():
                l.bias.fill_(0.05)
    p = _deepfm_params(models[0], np.concatenate([m.table_shard.cpu().numpy() for m in models]).astype(np.float64))
    for step in range(2):
        batches, labels = [], []
        for r in range(world):
            ids = np.stack([rng.integers(0, v, B) for v in vocabs], 1).astype(np.int32)
            ids[:4, 2] = 0  # repeated rows within and across ranks
            if dedup:
                ids[:, 7] = rng.integers(0, 3, B)  # a field of a few hot rows
            batches.append((torch.as_tensor(rng.random((B, nd)), dtype=torch.float32, device=gpu),
                            torch.as_tensor(ids, device=gpu)))
            labels.append(torch.as_tensor(rng.integers(0, 2, B), dtype=torch.float32, device=gpu))
        off = models[0]._dropout().offset
        if world == 1:
            losses = [models[0].train_step(batches[0], labels[0], lr=lr, return_loss=True,
                                           dropout=None if drop else False)]
        else:
            losses = _simulated_deepfm_train(models, batches, labels, lr, 0.2 if drop else 0.0)
        cat = lambda xs: np.concatenate([x.cpu().numpy() for x in xs])
        masks = _global_masks(9, world, off, B, [64, 32], 0.2) if drop else None
        p, ce = O.deepfm_train_step(cat([b_[0] for b_ in batches]), cat([b_[1] for b_ in batches]), cat(labels), p,
                                    lr, rw, rv, nd=nd, masks=masks)
        assert_scaled_close(cat(losses), ce, what=f"step {step} loss")
        full = np.concatenate([m.table_shard.cpu().numpy() for m in models])
        assert_scaled_close(full, np.concatenate(p["tables"]), what=f"step {step} tables")
        for r, m in enumerate(models):
            mine = _deepfm_params(m, full)
            for name in ("w1", "v"):
                assert_scaled_close(mine[name], p[name], what=f"step {step} rank {r} {name}")
            for li, ((W_, b_), (Wr, br)) in enumerate(zip(mine["dnn_hidden"] + [mine["dnn_out"]],
                                                        p["dnn_hidden"] + [p["dnn_out"]])):
                assert_scaled_close(W_, Wr, what=f"step {step} rank {r} W{li}")
                assert_scaled_close(b_, br, what=f"step {step} rank {r} b{li}")
            # w0 moves by -lr * sum_b g_b (|g_b| <= 1/(world B)): fp32 error ~ lr, not |w0|
            w0, r0 = float(mine["w0"].reshape(-1)[0]), float(np.asarray(p["w0"]).reshape(-1)[0])
            assert abs(w0 - r0) <= 1e-5 * max(abs(r0), lr * (step + 1)), (step, w0, r0)
    for m in models:
        assert int(m.ops.err.item()) == 0


def _check_dedup_route(sh, ids, cap, send, slot_of):
    """What the dedup route promises, whatever order it numbers the distinct
    rows in: owner o's words [0, n_o) are n_o = min(distinct, cap) distinct
    local rows it owns (all of them when they fit), the rest -1; every lookup's
    slot holds its own row (-1 only past the capacity).  Returns overflow."""
    rpr, world = sh.rows_per_rank, sh.world
    rows = (sh.offsets.cpu().numpy()[None, :] + ids.astype(np.int64)).reshape(-1)
    owner = np.minimum(rows // rpr, world - 1)
    send = send.astype(np.int64)
    slot = slot_of.reshape(-1).astype(np.int64)
    over = False
    for o in range(world):
        need = np.unique(rows[owner == o])
        n_o = min(need.size, cap)
        words = send[o * cap:(o + 1) * cap]
        assert np.all(words[n_o:] == -1)
        got = words[:n_o] + o * rpr
        assert np.unique(got).size == n_o and np.isin(got, need).all()
        over |= need.size > cap
        mine = owner == o
        ok = slot[mine] >= 0
        assert need.size > cap or ok.all()
        s = slot[mine][ok]
        assert np.all(s // cap == o)
        np.testing.assert_array_equal(send[s] + o * rpr, rows[mine][ok])
    return over


@pytest.mark.gpu
@pytest.mark.parametrize("world,cap_frac,B", [(1, 1.0, 256), (3, 1.0, 256), (8, 1.0, 4096), (8, 0.05, 256),
                                               (2, 1.0, 3000), (1, 1.0, 4096), (2, 1.0, 17000)])
def test_gpu_dedup_route_matches_reference(gpu, world, cap_frac, B):
    """rs_shard_dedup_route == the numpy double (distinct rows per owner in
    row order, slot_of, -1 padding), Zipf-like ids with many repeats; a
    capacity below the distinct count raises the overflow flag; then the
    forward through the deduplicated exchange (simulated world) equals
    O.deepfm.  B <= 4096: the per-field hash path (rows numbered by first
    occurrence: checked by what the route promises, and run twice for
    determinism); 17000: the device-wide radix sort (row order: equal to the
    numpy double word for word)."""
    from recommender_system_amd.sharded import ShardedDeepFM
    from tests.helpers import assert_rel_close
    rng = np.random.default_rng(world * 5 + 3)
    vocabs = [int(v) for v in rng.integers(1, 3000, 26)]
    k, nd = 16, 13
    cols = _deepfm_columns(vocabs, nd, k)
    models = [ShardedDeepFM(cols, 10, 1e-4, 1e-4, [64, 32], 1, "relu", embed_dim=k, device=gpu, seed=4,
                            world=world, rank=r, dedup=cap_frac) for r in range(world)]
    cpu = CpuOps()
    batches = []
    for r, m in enumerate(models):
        ids = np.minimum(rng.zipf(1.3, size=(B, 26)) - 1, np.array(vocabs) - 1).astype(np.int32)
        batches.append((torch.rand(B, nd, device=gpu), torch.as_tensor(ids, device=gpu)))
        rb = m._rbufs(B)
        m.route(batches[-1][1], rb)
        ref = {"cap": rb["cap"], "send": torch.empty(rb["n"], dtype=torch.int32),
               "slot_of": torch.empty(B, 26, dtype=torch.int32)}
        cpu.dedup_route(m.emb, torch.as_tensor(ids), ref)
        over = bool(m.ops.overflow_flag(rb).item())
        assert over == bool(getattr(cpu, "dedup_overflow", False)), (over, cap_frac)
        cpu.dedup_overflow = False
        send, slot_of = rb["send"].cpu().numpy(), rb["slot_of"].cpu().numpy()
        assert _check_dedup_route(m.emb, ids, rb["cap"], send, slot_of) == over
        if B > 4096:
            np.testing.assert_array_equal(send, ref["send"].numpy())
            np.testing.assert_array_equal(slot_of, ref["slot_of"].numpy())
        else:
            m.route(batches[-1][1], rb)
            m.ops.overflow_flag(rb)
            np.testing.assert_array_equal(rb["send"].cpu().numpy(), send)
            np.testing.assert_array_equal(rb["slot_of"].cpu().numpy(), slot_of)
        if cap_frac < 0.1:
            assert over
    if cap_frac >= 0.1:
        outs = _simulated_deepfm_step(models, batches)
        for r in range(world):
            ref = _compact_deepfm_reference(models, batches[r][0].cpu().numpy(), batches[r][1].cpu().numpy())
            assert_rel_close(outs[r], ref, what=f"rank {r}")
        # fewer rows on the wire than the field-range records whenever ids
        # repeat (the capacity itself is rounded up to 64 words per owner)
        for m in models:
            assert int((m._rbufs(B)["send"] >= 0).sum().item()) < B * 26
    for m in models:
        assert int(m.ops.err.item()) == 0


@pytest.mark.gpu
def test_gpu_dedup_unchecked_overflow_leaves_no_stale_flags(gpu):
    """An unchecked forward (check=False) whose distinct rows overflow a small
    dedup capacity leaves the overflow and id flags set; the next checked
    forward restarts both, so it neither raises a false IndexError nor takes
    the fallback, and equals the exact forward."""
    from recommender_system_amd.sharded import ShardedDeepFM
    from tests.helpers import assert_rel_close
    rng = np.random.default_rng(31)
    vocabs = [int(v) for v in rng.integers(500, 3000, 26)]
    m = ShardedDeepFM(_deepfm_columns(vocabs, 13, 16), 10, 1e-4, 1e-4, [64, 32], 1, "relu", embed_dim=16,
                      device=gpu, seed=3, world=1, rank=0, dedup=0.05)
    m.force_rows = True
    B = 512
    wide = torch.as_tensor(np.stack([rng.integers(0, v, B) for v in vocabs], 1).astype(np.int32), device=gpu)
    dense = torch.rand(B, 13, device=gpu)
    m.forward((dense, wide), check=False)
    torch.cuda.synchronize()
    assert int(m._rbufs(B)["overflow"].item()) > 0  # slot -1 lookups (they also set the id flag)
    few = torch.zeros(B, 26, dtype=torch.int32, device=gpu)  # one distinct row per field: fits
    got = m.forward((dense, few)).clone()
    assert int(m.ops.err.item()) == 0
    m2 = ShardedDeepFM(_deepfm_columns(vocabs, 13, 16), 10, 1e-4, 1e-4, [64, 32], 1, "relu", embed_dim=16,
                       device=gpu, seed=3, world=1, rank=0)
    m2.force_rows = True
    exp = m2.forward((dense, few))
    assert_rel_close(got.cpu().numpy(), exp.cpu().numpy(), what="checked dedup forward after an overflow")


@pytest.mark.gpu
def test_gpu_forward_stream_after_unchecked_bad_ids(gpu):
    """An unchecked forward with out-of-range ids leaves the sticky id flag
    set; a following checked forward_stream (ShardedDeepFM and the sharded
    FM) restarts it, so valid batches neither raise a false IndexError nor
    change their outputs (forward_stream checked a stale flag)."""
    from recommender_system_amd.sharded import ShardedDeepFM, ShardedEmbeddingFM
    rng = np.random.default_rng(41)
    vocabs = [int(v) for v in rng.integers(50, 400, 26)]
    m = ShardedDeepFM(_deepfm_columns(vocabs, 13, 16), 10, 1e-4, 1e-4, [64, 32], 1, "relu", embed_dim=16,
                      device=gpu, seed=4, world=1, rank=0)
    m.force_rows = True
    B = 128
    dense = torch.rand(B, 13, device=gpu)
    bad = torch.full((B, 26), 10 ** 6, dtype=torch.int32, device=gpu)
    m.forward((dense, bad), check=False)
    torch.cuda.synchronize()
    assert int(m.ops.err.item()) != 0
    ok = torch.as_tensor(np.stack([rng.integers(0, v, B) for v in vocabs], 1).astype(np.int32), device=gpu)
    outs = m.forward_stream([(dense, ok), (dense, ok)], check=True)
    exp = m.forward((dense, ok))
    for o in outs:
        assert torch.equal(o, exp)
    sh = ShardedEmbeddingFM(vocabs, 16, 13, 10, device=gpu, seed=4, world=1, rank=0)
    sh.forward(dense, bad, check=False)
    torch.cuda.synchronize()
    assert int(sh.ops.err.item()) != 0
    souts = sh.forward_stream([(dense, ok)], check=True)
    assert torch.equal(souts[0], sh.forward(dense, ok))


def test_raise_flag_keeps_the_flag_bits():
    """A layout flag (RS_FLAG_LAYOUT) raises RSError, a bad id IndexError, 0
    nothing (the sharded checks reported a layout error as a bad
    id)."""
    from recommender_system_amd import _lib
    from recommender_system_amd.sharded import raise_flag
    raise_flag(torch.zeros(1, dtype=torch.int32), "t")
    with pytest.raises(IndexError):
        raise_flag(torch.tensor([_lib.FLAG_BAD_ID]), "t")
    for bits in (_lib.FLAG_LAYOUT, _lib.FLAG_LAYOUT | _lib.FLAG_BAD_ID):
        with pytest.raises(_lib.RSError, match="LAYOUT"):
            raise_flag(torch.tensor([bits]), "t")


def _flag_or_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from recommender_system_amd import _lib
    from recommender_system_amd.sharded import raise_flag
    try:
        # rank 0 saw a bad id, rank 1 a layout error: every rank must see both
        f = torch.tensor([_lib.FLAG_BAD_ID if rank == 0 else _lib.FLAG_LAYOUT], dtype=torch.int32)
        try:
            raise_flag(f, "t", group=None, world=world)
            q.put((rank, "no raise"))
        except _lib.RSError as e:
            q.put((rank, str(e)))
        except IndexError as e:
            q.put((rank, "IndexError " + str(e)))
    finally:
        dist.destroy_process_group()


def test_raise_flag_ors_the_bits_across_ranks():
    """the ranks' flag masks were reduced by MAX (BAD_ID 1 + LAYOUT
    2 -> 2, the bad id lost); they are OR-ed now — every rank raises RSError
    naming both bits (gloo, world 2)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_flag_or_worker, args=(r, 2, port, q)) for r in range(2)]
    for p_ in procs:
        p_.start()
    res = sorted(q.get(timeout=120) for _ in range(2))
    for p_ in procs:
        p_.join(timeout=60)
        assert p_.exitcode == 0
    for rank, msg in res:
        assert "RS_FLAG_BAD_ID" in msg and "RS_FLAG_LAYOUT" in msg, (rank, msg)


@pytest.mark.gpu
def test_gpu_sharded_deepfm_pipelined(gpu):
    """ShardedDeepFM.forward_stream / pipe_step (batch t+1's route + owner
    gather on a side stream beside batch t's rs_deepfm_fwd, two buffer
    slots, hub fork / join) == the per-batch forward bit for bit, eager and
    replayed from a hipGraph; world 1 with the row protocol forced."""
    from recommender_system_amd.sharded import ShardedDeepFM
    rng = np.random.default_rng(5)
    vocabs = [int(v) for v in rng.integers(1, 400, 26)]
    m = ShardedDeepFM(_deepfm_columns(vocabs, 13, 16), 10, 1e-4, 1e-4, [64, 32], 1, "relu", embed_dim=16,
                      device=gpu, seed=9, world=1, rank=0)
    m.force_rows = True
    B, T = 300, 4
    batches = [(torch.rand(B, 13, device=gpu),
                torch.as_tensor(np.stack([rng.integers(0, v, B) for v in vocabs], 1).astype(np.int32), device=gpu))
               for _ in range(T)]
    ref = [m.forward(b).clone() for b in batches]
    for o, r in zip(m.forward_stream(batches), ref):
        assert torch.equal(o, r)
    outs = [torch.full((B, 1), 7.0, device=gpu) for _ in range(T)]
    m.pipe_prologue(batches[0][1], 0)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for t in range(T):
                m.pipe_step((batches[t][0], outs[t], t % 2), (batches[t + 1][1], (t + 1) % 2) if t + 1 < T else None)
    torch.cuda.current_stream().wait_stream(s)
    m.pipe_prologue(batches[0][1], 0)
    g.replay()
    torch.cuda.synchronize()
    for o, r in zip(outs, ref):
        assert torch.equal(o, r)
    assert int(m.ops.err.item()) == 0
