"""Row-sharded embedding lookup + FM across the GPUs of one node.

The reference has no distributed code.  This is the MI355X-native design for
BASELINE config 5: ONE concatenated embedding table (global row of (b,c) =
field_offsets[c] + id) split into contiguous row blocks, one per rank
(owner = row // rows_per_rank); dense parameters (w0, w1, v) replicated.
Per step and rank (B local samples, data parallel):

  1. rs_shard_slot_bucketize -> every lookup gets a slot in a fixed-capacity
                               per-owner message (cap = 1.15 n/world + 64,
                               stable, deterministic); local row ids to request
  2. all_to_all(slots)      -> the row ids every peer asks of me    (RCCL)
  3. rs_gather_rows         -> serve them from my shard (-1 -> zero row)
  4. all_to_all(rows)       -> my lookups' rows, slot-addressed     (RCCL)
  5. rs_embed_fm_fwd        -> FM logit straight from the exchange buffer
                               (ids = slot of each lookup: the headline kernel)

Equal, host-known splits: no host synchronisation inside the step, so the
whole step is enqueued asynchronously.  A slot overflow (an owner receiving
more than cap lookups from one rank: ~20 sigma for uniform ids) raises a
device flag; ``forward(check=True)`` then recomputes the step with the exact
protocol (``lookup``: counts all-to-all, one host sync, variable splits,
rs_shard_bucketize / rs_unpermute_rows / rs_rows_fm_fwd), so the result is
always exact.

Collectives go through torch.distributed (backend "nccl" = RCCL over xGMI on
ROCm; "gloo" in the CPU tests).  On an 8-GPU MI355X node every peer pair has
its own xGMI link, so all-to-all is per-link bound: at B=4096, F=26, k=16,
world=8 each peer exchange is ~13.3k ids (53 KB) and ~13.3k rows (852 KB).
No all-reduce: forward only.  The local ops are pluggable (``ops``) so the
exchange protocol is testable with world_size>1 on CPU (tests/test_sharded_gloo.py).
"""
from __future__ import annotations

import ctypes as C
import math

import torch
import torch.distributed as dist

from . import _lib
from ._lib import call, ptr


_FLAG_BITS = 8  # rs_flag bits carried across ranks


def raise_flag(f, what, group=None, world=1):
    """Raise for the rs_flag bits in the device flag `f` (OR-ed over the group
    first when world > 1 — one 0/1 word per bit reduced by MAX, since MAX of
    the masks is not their OR — so every rank sees every bit and takes the
    same branch): RS_FLAG_LAYOUT / RS_FLAG_TIMEOUT (or any unknown bit) ->
    RSError, RS_FLAG_BAD_ID alone -> IndexError (TF's InvalidArgumentError on
    an out-of-range Embedding id)."""
    if world > 1:
        per_bit = torch.stack([(f.reshape(-1)[0] >> i) & 1 for i in range(_FLAG_BITS)])
        dist.all_reduce(per_bit, op=dist.ReduceOp.MAX, group=group)
        f = (per_bit << torch.arange(_FLAG_BITS, device=per_bit.device, dtype=per_bit.dtype)).sum()
    bits = int(f.item())
    if bits & ~_lib.FLAG_BAD_ID:
        raise _lib.RSError(f"{what}: device error flag {bits:#x} ({_lib.flag_names(bits)})")
    if bits:
        raise IndexError(f"{what}: embedding id out of range")


class _DevBuf:
    """A device allocation as a torch tensor view (__cuda_array_interface__)."""

    def __init__(self, ptr_, nbytes):
        self.__cuda_array_interface__ = {"shape": (int(nbytes),), "typestr": "|u1", "data": (int(ptr_), False),
                                         "version": 3, "strides": None}


class PeerExchange:
    """Equal-split all-to-all over hipIpc-mapped mailboxes (rs_peer_a2a,
    csrc/peer.hip) — the RCCL all-to-all's drop-in for the sharded lookup's
    fixed-size record exchanges.  Every rank allocates one uncached mailbox
    ([world][block_bytes] data + ready / full step flags), exports its IPC
    handle, and opens every peer's (handles all-gathered over the group once,
    before any timed step).  ``all_to_all(send)`` is ONE launch: each rank
    writes its block for peer p straight into p's mailbox (xGMI stores on an
    8-GPU node) once p has said its mailbox is free for the step, flags it, and
    the launch ends when every block of the step is in its own mailbox — the
    returned tensor (a view of the mailbox) is then valid until the next
    ``all_to_all`` on this exchange.  Step numbers live on the device, so the
    call is graph-capturable.  Every wait is bounded: a timeout raises
    RS_FLAG_TIMEOUT in ``err`` (check with ``check()``).

    Requires every rank's process to see every peer's device (one node) and
    the HIP dmabuf IPC path (HSA_ENABLE_IPC_MODE_LEGACY=0).  Tested with two
    processes on one device (tests/test_peer_exchange.py); RCCL stays the
    default exchange.  At world 1 with the lean ordering the mailbox is
    ordinary device memory (no peer maps it)."""

    def __init__(self, block_bytes, group=None, world=None, rank=None, device=None, chunks=None,
                 spin_limit=1 << 24):
        self.group = group
        self.world = int(world) if world is not None else dist.get_world_size(group)
        self.rank = int(rank) if rank is not None else dist.get_rank(group)
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        self.block_bytes = int(block_bytes)
        if self.block_bytes % 16:
            raise ValueError("PeerExchange: block_bytes must be a multiple of 16")
        lib = _lib.lib()
        self.mbox_bytes = int(lib.rs_peer_mailbox_bytes(self.world, self.block_bytes))
        if self.mbox_bytes < 0:
            raise ValueError("PeerExchange: bad world / block size")
        # Setup is collective and fails collectively: a rank whose allocation,
        # export or mapping fails still takes part in every collective below,
        # and then every rank raises (no rank is left waiting in a collective).
        self._mine, self._opened, self._local = None, [], None
        h = (C.c_uint8 * 64)()
        err = ""
        # world 1 (the bench's forced self-exchange): no peer maps the mailbox
        # and nothing crosses a device, so it is ordinary (cached) device
        # memory written with plain stores under the lean ordering
        # (RS_OPT_PEER_FENCES 0; peer.hpp) instead of uncached memory
        local = self.world == 1 and _lib.lib().rs_get_option(_lib.OPT_PEER_FENCES) == 0
        try:
            if local:
                self._local = torch.zeros(self.mbox_bytes, dtype=torch.uint8, device=self.device)
            else:
                mine = C.c_void_p()
                call("rs_peer_alloc", self.mbox_bytes, C.addressof(mine))
                self._mine = mine.value
                call("rs_peer_ipc_handle", self._mine, C.addressof(h))
        except Exception as e:  # noqa: BLE001 — reported collectively below
            err = f"rank {self.rank}: {e}"
        # every rank's [ok | handle (64 B)] — over the group's backend (gloo: CPU tensors)
        cpu = dist.get_backend(group) == "gloo"
        ht = torch.tensor([0 if err else 1] + list(bytes(h)), dtype=torch.uint8, device="cpu" if cpu else self.device)
        allh = [torch.empty_like(ht) for _ in range(self.world)]
        dist.all_gather(allh, ht, group=group)
        allh = [a.cpu() for a in allh]
        ptrs = []
        if all(int(a[0]) == 1 for a in allh):
            try:
                for r in range(self.world):
                    if r == self.rank:
                        ptrs.append(self._mine if self._local is None else self._local.data_ptr())
                        continue
                    hr = (C.c_uint8 * 64)(*allh[r][1:].tolist())
                    pr = C.c_void_p()
                    call("rs_peer_ipc_open", C.addressof(hr), C.addressof(pr))
                    self._opened.append(pr.value)
                    ptrs.append(pr.value)
            except Exception as e:  # noqa: BLE001
                err = err or f"rank {self.rank}: {e}"
        else:
            err = err or "a peer failed to allocate / export its mailbox"
        okt = torch.tensor([0 if err else 1], dtype=torch.int32, device="cpu" if cpu else self.device)
        dist.all_reduce(okt, op=dist.ReduceOp.MIN, group=group)
        if int(okt.item()) != 1:
            for p_ in self._opened:
                _lib.lib().rs_peer_ipc_close(p_)
            self._opened = []
            dist.barrier(group=group)
            if self._mine:
                _lib.lib().rs_peer_free(self._mine)
                self._mine = None
            raise _lib.RSError(f"PeerExchange setup failed ({err or 'on another rank'})")
        self.mailboxes = torch.tensor(ptrs, dtype=torch.int64, device=self.device)
        self.state = torch.zeros(int(lib.rs_peer_state_bytes()), dtype=torch.uint8, device=self.device)
        self.err = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.recv = (self._local[:self.world * self.block_bytes] if self._local is not None else
                     torch.as_tensor(_DevBuf(self._mine, self.world * self.block_bytes), device=self.device))
        if chunks is None:  # ~256 workgroups in all, at least 1 per destination
            chunks = max(1, min(1024 // self.world, 256 // self.world, -(-self.block_bytes // 16384)))
        self.chunks = int(chunks)
        self.spin_limit = int(spin_limit)
        torch.cuda.synchronize(self.device)
        dist.barrier(group=group)  # every mailbox opened before any rank writes

    def all_to_all(self, send):
        """send: contiguous device tensor of world * block_bytes bytes (block p
        for rank p); returns the mailbox view (uint8, world * block_bytes)."""
        if send.numel() * send.element_size() != self.world * self.block_bytes or not send.is_contiguous():
            raise ValueError("PeerExchange.all_to_all: send must be contiguous, world * block_bytes bytes")
        call("rs_peer_a2a", ptr(send), self.block_bytes, ptr(self.mailboxes), self.rank, self.world, ptr(self.state),
             self.chunks, self.spin_limit, ptr(self.err), _lib.stream())
        return self.recv

    def gather_all_to_all(self, ids, nw, table, err=None):
        """The owner's row service fused with the exchange: block p = the
        64-B rows table[ids[p][i]] (i < nw; -1 = zero row) of this rank's
        shard, written straight into peer p's mailbox (rs_peer_gather_a2a;
        block_bytes must be nw * 64).  Returns the mailbox view."""
        if self.block_bytes != nw * 64 or table.shape[1] != 16 or ids.numel() < self.world * nw:
            raise ValueError("PeerExchange.gather_all_to_all: block_bytes != nw * 64 or k != 16")
        call("rs_peer_gather_a2a", ptr(ids), nw, ptr(table), table.shape[0], 16, ptr(self.mailboxes), self.rank,
             self.world, ptr(self.state), self.chunks, self.spin_limit, ptr(err if err is not None else self.err),
             _lib.stream())
        return self.recv

    def check(self, what="PeerExchange"):
        v = int(self.err.item())
        if v:
            self.err.zero_()
            raise _lib.RSError(f"{what}: device error flag {v:#x} ({_lib.flag_names(v)})")

    def close(self):
        """Collective: every rank stops writing before any mailbox is unmapped or freed."""
        torch.cuda.synchronize(self.device)
        dist.barrier(group=self.group)
        for p_ in self._opened:
            _lib.lib().rs_peer_ipc_close(p_)
        self._opened = []
        dist.barrier(group=self.group)
        if self._mine:
            _lib.lib().rs_peer_free(self._mine)
            self._mine = None
        self._local = None


class HipShardOps:
    """Local per-rank steps on librs_hip.so kernels."""

    def __init__(self, device):
        self.device = device
        self.err = torch.zeros(1, dtype=torch.int32, device=device)
        self._ws = None

    def bucketize(self, ids, offsets, vocab, rows_per_rank, world):
        B, F = ids.shape
        n = B * F
        counts = torch.empty(world, dtype=torch.int32, device=self.device)
        perm = torch.empty(n, dtype=torch.int32, device=self.device)
        send_rows = torch.empty(n, dtype=torch.int32, device=self.device)
        wsz = _lib.lib().rs_shard_workspace_size(n, world)
        if self._ws is None or self._ws.numel() < wsz:
            self._ws = torch.zeros(wsz, dtype=torch.uint8, device=self.device)  # zeroed once (rs_capi.h)
        call("rs_shard_bucketize", ptr(ids), _lib.id_kind(ids), ids.stride(0), ptr(offsets), ptr(vocab), F, B,
             rows_per_rank, world, ptr(counts), ptr(perm), ptr(send_rows), ptr(self._ws), ptr(self.err),
             _lib.stream())
        return counts, perm, send_rows

    def slot_bucketize(self, ids, offsets, vocab, rows_per_rank, world, cap, bufs):
        B, F = ids.shape
        n = B * F
        if bufs.get("ws_n") != (n, world):
            wsz = _lib.lib().rs_shard_workspace_size(n, world)
            if self._ws is None or self._ws.numel() < wsz:
                self._ws = torch.zeros(wsz, dtype=torch.uint8, device=self.device)  # zeroed once (rs_capi.h)
            bufs["ws_n"] = (n, world)
        call("rs_shard_slot_bucketize", ptr(ids), _lib.id_kind(ids), ids.stride(0), ptr(offsets), ptr(vocab), F, B,
             rows_per_rank, world, cap, ptr(bufs["counts"]), ptr(bufs["slot_of"]), ptr(bufs["send"]), ptr(self._ws),
             ptr(self.err), ptr(bufs["overflow"]), _lib.stream())
        return bufs["slot_of"], bufs["send"]

    def gather_rows_into(self, table, rows, out):
        call("rs_gather_rows", ptr(table), table.shape[0], table.shape[1], ptr(rows), rows.numel(), ptr(out),
             ptr(self.err), _lib.stream())
        return out

    def slots_fm(self, got, slot_of, dense, n_fields, k, prepared, w0, kfm, bufs, out=None):
        """FM logit with lookup (b, c)'s row at got[slot_of[b*F + c]]: the
        headline kernel with ids = slots, zero field offsets, vocab = #slots."""
        B = dense.shape[0]
        logit = out if out is not None else torch.empty(B, 1, dtype=torch.float32, device=self.device)
        call("rs_embed_fm_fwd", ptr(slot_of), _lib.ID_I32, n_fields, ptr(dense), dense.stride(0), dense.shape[1],
             ptr(got), ptr(bufs["zoff"]), ptr(bufs["nslots"]), n_fields, k, ptr(prepared), ptr(w0), kfm, ptr(logit),
             None, B, ptr(bufs["overflow"]), _lib.stream())
        return logit

    def flags(self, bufs):
        """[rs_flag bits of the id flag, slot overflow seen] (device tensor; resets)."""
        v = torch.stack([self.err[0], bufs["overflow"][0].clamp(max=1)])
        self.err.zero_()
        bufs["overflow"].zero_()
        return v

    def gather_rows(self, table, rows):
        out = torch.empty(rows.numel(), table.shape[1], dtype=torch.float32, device=self.device)
        call("rs_gather_rows", ptr(table), table.shape[0], table.shape[1], ptr(rows), rows.numel(), ptr(out),
             ptr(self.err), _lib.stream())
        return out

    def unpermute(self, src, perm):
        out = torch.empty(perm.numel(), src.shape[1], dtype=torch.float32, device=self.device)
        call("rs_unpermute_rows", ptr(src), ptr(perm), src.shape[1], perm.numel(), ptr(out), _lib.stream())
        return out

    def rows_fm(self, emb, dense, n_fields, k, prepared, w0, kfm):
        B = dense.shape[0]
        logit = torch.empty(B, 1, dtype=torch.float32, device=self.device)
        call("rs_rows_fm_fwd", ptr(emb), ptr(dense), dense.stride(0), dense.shape[1], n_fields, k, ptr(prepared),
             ptr(w0), kfm, ptr(logit), B, _lib.stream())
        return logit

    # -- partial protocol (rs_shard_field_route / rs_shard_owner_fm / rs_shard_fm_combine)
    # Record layouts (in 4-byte words): row-id records of `rec` words, slot j
    # at word j; partial records `pst` words apart starting at word `poff` of
    # the buffer (separate buffers: rec = S, poff = 0, pst = P; the pipelined
    # fused buffer: rec = pst = S + P, poff = S).
    def field_route(self, sh, ids, send, rec=None):
        B, F = ids.shape
        call("rs_shard_field_route", ptr(ids), _lib.id_kind(ids), ids.stride(0), ptr(sh.offsets), ptr(sh.vocab), F, B,
             sh.rows_per_rank, sh.world, ptr(sh.owner_fields), sh.slot_stride, rec or sh.slot_stride, ptr(send),
             ptr(self.err), _lib.stream())
        return send

    def owner_partials(self, sh, recv, n_pairs, out, rec=None, poff=0, pst=None):
        lo, n_own = sh.owner_field_ranges[sh.rank]
        call("rs_shard_owner_fm", ptr(recv), rec or sh.slot_stride, lo, n_own, ptr(sh.table_shard),
             sh.table_shard.shape[0], sh.nd, sh.F, sh.k, ptr(sh.prepared), sh.kfm, ptr(out) + 4 * poff,
             pst or sh.partial_width, n_pairs, ptr(self.err), _lib.stream())
        return out

    def combine(self, sh, partials, dense, out, poff=0, pst=None):
        B = dense.shape[0]
        call("rs_shard_fm_combine", ptr(partials) + 4 * poff, pst or sh.partial_width, sh.world, B, ptr(dense),
             dense.stride(0), dense.shape[1], sh.F, sh.k, ptr(sh.prepared), ptr(sh.w0), sh.kfm, ptr(out),
             _lib.stream())
        return out

    def pipe(self, sh, recv, send, prev=None, cur=None, nxt=None):
        """rs_shard_fm_pipe: combine(prev) | owner(cur) | route(nxt) in ONE launch
        on the fused records (sharded.py pipe_step)."""
        lo, n_own = sh.owner_field_ranges[sh.rank]
        B = (cur if cur is not None else (prev[0] if prev is not None else nxt[1])).shape[0]
        if cur is None:
            n_own = 0  # no owner part this step (its partial words are never read)
        ids = nxt[1] if nxt is not None else None
        call("rs_shard_fm_pipe", ptr(recv), lo, n_own, ptr(sh.table_shard), sh.table_shard.shape[0],
             ptr(prev[0]) if prev is not None else None, prev[0].stride(0) if prev is not None else 0,
             ptr(prev[1]) if prev is not None else None, ptr(ids), _lib.id_kind(ids) if ids is not None else 0,
             ids.stride(0) if ids is not None else 0, ptr(sh.offsets), ptr(sh.vocab), sh.rows_per_rank,
             ptr(sh.owner_fields), sh.slot_stride, ptr(send), sh.world, B, sh.nd, sh.F, sh.k, ptr(sh.prepared),
             ptr(sh.w0), sh.kfm, ptr(self.err), _lib.stream())

    def pipe_peer(self, sh, recv, send, xsend, xslot, exchange, ex, prev=None, cur=None, nxt=None, B=None):
        """rs_shard_fm_pipe_peer: E(t+1) (send slot xslot -> the peers'
        mailbox slot xslot, if ``exchange``) | combine(prev) | owner(cur) |
        route(nxt = ids) in ONE launch (sharded.py pipe2_step)."""
        lo, n_own = sh.owner_field_ranges[sh.rank]
        if cur is None:
            n_own = 0  # no owner part this step (its partial words are never read)
        call("rs_shard_fm_pipe_peer", ptr(recv), ptr(send), ptr(xsend), int(xslot), int(bool(exchange)), lo, n_own,
             ptr(sh.table_shard), sh.table_shard.shape[0], ptr(prev[0]) if prev is not None else None,
             prev[0].stride(0) if prev is not None else 0, ptr(prev[1]) if prev is not None else None, ptr(nxt),
             _lib.id_kind(nxt) if nxt is not None else 0, nxt.stride(0) if nxt is not None else 0, ptr(sh.offsets),
             ptr(sh.vocab), sh.rows_per_rank, ptr(sh.owner_fields), sh.slot_stride, sh.world, B, sh.nd, sh.F, sh.k,
             ptr(sh.prepared), ptr(sh.w0), sh.kfm, ptr(self.err), ptr(ex.mailboxes), sh.rank, ptr(ex.state),
             ex.chunks, ex.spin_limit, ptr(ex.err), _lib.stream())

    # -- training (ShardedEmbeddingFM.train_step)
    def combine_grad(self, sh, partials, dense, labels, scale, logit, gs, loss=None):
        B = dense.shape[0]
        call("rs_shard_fm_combine_grad", ptr(partials), sh.partial_width, sh.world, B, ptr(dense), dense.stride(0),
             dense.shape[1], sh.F, sh.k, ptr(sh.prepared), ptr(sh.w0), sh.kfm, ptr(labels), float(scale), ptr(logit),
             ptr(gs), gs.stride(0), ptr(loss), _lib.stream())

    def dense_grads(self, sh, dense, gs, grad):
        """The requester's FM parameter gradients: dense columns + dw0."""
        d, kfm, nd = sh.d, sh.kfm, sh.nd
        call("rs_fm_param_grads_strided", ptr(dense) if nd else None, dense.stride(0), ptr(gs), gs.stride(0),
             ptr(gs) + 4 * kfm, gs.stride(0), ptr(sh.v), dense.shape[0], nd, kfm, ptr(grad), ptr(grad) + 4 * d,
             ptr(grad) + 4 * d * (1 + kfm), _lib.stream())

    def owner_grads(self, sh, recv, gs_all, grad, lr, bufs):
        """Owner side: dL/drow of every owned lookup, this owner's part of the
        FM parameter gradients over its columns, and the row SGD."""
        lo, n_own = sh.owner_field_ranges[sh.rank]
        if n_own == 0:
            return
        n_pairs = gs_all.shape[0]
        d, kfm, k, S = sh.d, sh.kfm, sh.k, sh.slot_stride
        col = sh.nd + lo * k
        call("rs_shard_owner_fm_grad", ptr(recv), S, lo, n_own, ptr(sh.table_shard), sh.table_shard.shape[0], sh.nd,
             k, ptr(sh.w1), ptr(sh.v), kfm, ptr(gs_all), gs_all.stride(0), n_pairs, ptr(bufs["xo"]),
             ptr(bufs["drows"]), ptr(grad) + 4 * col, ptr(grad) + 4 * (d + col * kfm), _lib.stream())
        call("rs_embedding_sgd", ptr(sh.table_shard), sh.table_shard.shape[0], k, ptr(recv), _lib.ID_I32, S,
             ptr(bufs["zoff"]), ptr(bufs["svocab"]), n_own, n_pairs, ptr(bufs["drows"]), n_own * k, float(lr),
             ptr(bufs["ws"]), None, _lib.stream())

    def apply(self, sh, grad, lr, reg_w, reg_v):
        d, kfm, st = sh.d, sh.kfm, _lib.stream()
        g = ptr(grad)
        _lib.sgd_update_multi([(sh.w1, g, d, reg_w), (sh.v, g + 4 * d, d * kfm, reg_v),
                               (sh.w0, g + 4 * d * (1 + kfm), 1, 0.0)], lr, st)
        sh.prepare()

    # -- row protocol of ShardedDeepFM (rs_shard_row_route / rs_gather_rows / rs_deepfm_fwd)
    def row_route(self, sh, ids, send, slot_of):
        B, F = ids.shape
        call("rs_shard_row_route", ptr(ids), _lib.id_kind(ids), ids.stride(0), ptr(sh.offsets), ptr(sh.vocab), F,
             B, sh.rows_per_rank, sh.world, ptr(sh.owner_fields), sh.slot_stride, ptr(send), ptr(slot_of),
             ptr(self.err), _lib.stream())
        return send, slot_of

    def deepfm_rows(self, model, got, rb, dense, out):
        """DeepFM forward with lookup (b, c)'s row at got[slot_of[b, c]]."""
        hm = rb.get("hmeta")
        if hm is None:  # the exchange layout's metadata on the host: offsets 0, n slots per field
            F = model.F
            hm = rb["hmeta"] = ((C.c_int64 * F)(*([0] * F)), (C.c_int64 * F)(*([int(rb["n"])] * F)))
        return _hip_deepfm(self, model, rb["slot_of"], got, rb["zoff"], rb["nslots"], dense, out, hm)

    def deepfm_table(self, model, ids, dense, out):
        """World 1: the DeepFM forward on the (whole-table) shard itself."""
        sh = model.emb
        return _hip_deepfm(self, model, ids, sh.table_shard, sh.offsets, sh.vocab, dense, out,
                           (sh.host_offsets, sh.host_vocab))

    # -- training of ShardedDeepFM (row protocol + reverse row exchange)
    def deepfm_grads(self, model, got, rb, dense, labels, scale, tb, loss, drop=None):
        """This rank's share of the DeepFM step: x = [dense | rows from the
        exchange buffer] (rs_embed_gather with ids = slot_of), forward with
        saved activations (rs_dense_fwd, rs_fm_fwd, s = x@v on rs_gemm),
        g = scale (sigmoid(z) - t) (rs_head_grad_scaled, scale = 1/(world B)),
        the DNN backward (split-K rs_gemm, rs_col_sum) and the FM gradients
        (rs_fm_x_grad, rs_fm_param_grads) into the views of tb's flat
        gradient; returns dL/dx [B, d].  drop = (_Dropout, rate, offsets):
        DNNLayer's Dropout draws of the hidden layers (rs_dropout), reused in
        the backward."""
        from .models import _dnn_backward
        sh, st = model.emb, _lib.stream()
        B, d, kfm = dense.shape[0], sh.d, sh.kfm
        x = tb["x"]
        call("rs_embed_gather", ptr(rb["slot_of"]), _lib.ID_I32, model.F, ptr(dense), dense.stride(0), model.nd,
             ptr(got), ptr(rb["zoff"]), ptr(rb["nslots"]), model.F, model.k, ptr(x), d, B, ptr(self.err), st)
        dnn = model.dnn
        layers = list(dnn.hidden_layer) + [dnn.output_layer]
        acts = [x]
        for i, layer in enumerate(dnn.hidden_layer):
            a = layer(acts[-1])
            if drop is not None:
                drop[0].redraw(a, drop[1], drop[2][i], st)
            acts.append(a)
        dnn_out = dnn.output_layer(acts[-1])
        fm_out = tb["fm"]
        # FMLayer on the dense x: its own packed image (nd = d, no fields)
        call("rs_fm_prepare", ptr(sh.w1), ptr(sh.v), d, 0, 0, kfm, ptr(tb["fm_prep"]), st)
        call("rs_fm_fwd", ptr(x), d, d, ptr(tb["fm_prep"]), ptr(sh.w0), kfm, ptr(fm_out), B, st)
        gw = (ptr(tb["gemm_ws"]), tb["gemm_ws"].numel())
        s = tb["s"]
        call("rs_gemm", 0, 0, B, kfm, d, 1.0, ptr(x), d, ptr(sh.v), kfm, 0.0, ptr(s), kfm, None, 0, *gw, st)
        g_fm, g_dnn = tb["g_fm"], tb["g_dnn"]
        call("rs_head_grad_scaled", ptr(fm_out), ptr(dnn_out), ptr(labels), B, 0.5, 0.5, float(scale), ptr(g_fm),
             ptr(g_dnn), ptr(loss), st)
        emp = lambda *shape: torch.empty(*shape, dtype=torch.float32, device=self.device)
        _, dx = _dnn_backward(layers, acts, g_dnn.view(B, 1), gw, emp, st, outs=tb["dnn_views"], drop=drop)
        call("rs_fm_x_grad", ptr(x), d, ptr(s), ptr(sh.w1), ptr(sh.v), B, d, kfm, ptr(g_fm), ptr(dx), d, st)
        call("rs_fm_param_grads", ptr(x), d, ptr(s), ptr(sh.v), B, d, kfm, ptr(g_fm), ptr(tb["dw1"]), ptr(tb["dv"]),
             ptr(tb["dw0"]), st)
        return dx

    def dedup_route(self, sh, ids, rb):
        """Distinct rows per owner (rs_shard_dedup_route): send words, slot_of."""
        B, F = ids.shape
        call("rs_shard_dedup_route", ptr(ids), _lib.id_kind(ids), ids.stride(0), ptr(sh.offsets), ptr(sh.vocab), F,
             B, sh.rows_per_rank, sh.world, rb["cap"], ptr(rb["send"]), ptr(rb["slot_of"]), ptr(rb["ws"]),
             ptr(self.err), ptr(rb["overflow"]), _lib.stream())
        return rb["send"], rb["slot_of"]

    def dedup_grads(self, model, dx, rb):
        """One gradient row per distinct row: the sum over its lookups."""
        B = dx.shape[0]
        call("rs_shard_dedup_grad", ptr(dx) + 4 * model.nd, dx.stride(0), model.F, model.k, B, model.world,
             ptr(rb["slot_of"]), ptr(rb["ws"]), ptr(rb["gsend"]), _lib.stream())
        return rb["gsend"]

    def overflow_flag(self, rb):
        """[distinct rows past the capacity seen] (device tensor; resets)."""
        v = rb["overflow"].clamp(max=1)
        rb["overflow"].zero_()
        return v

    def scatter_row_grads(self, model, dx, rb):
        """dL/drow of every lookup into its slot of the row-exchange layout."""
        call("rs_scatter_rows", ptr(dx) + 4 * model.nd, dx.stride(0), model.F, model.k, ptr(rb["slot_of"]),
             dx.shape[0], ptr(rb["gsend"]), _lib.stream())
        return rb["gsend"]

    def owner_row_sgd(self, model, recv, grecv, lr, tb, rec):
        """Owner: row-sparse SGD of the shard from the received row ids and
        their gradients, records of `rec` words (-1 words skipped; duplicates
        summed in record order: requester-major, then word order — the same
        on every rank)."""
        sh = model.emb
        n_pairs = recv.numel() // rec
        call("rs_embedding_sgd", ptr(sh.table_shard), sh.table_shard.shape[0], sh.k, ptr(recv), _lib.ID_I32, rec,
             ptr(tb["zoff"]), ptr(tb["svocab"]), rec, n_pairs, ptr(grecv), rec * sh.k, float(lr), ptr(tb["emb_ws"]),
             None, _lib.stream())

    def deepfm_apply(self, model, tb, lr):
        """SGD of the replicated parameters from the (all-reduced) flat
        gradient: l2(w_reg) on w1, l2(v_reg) on v (FMLayer), none elsewhere."""
        sh, st = model.emb, _lib.stream()
        upd = []
        for (L, _), (dW, db) in zip(tb["layers"], tb["dnn_views"]):
            upd += [(L.kernel, dW, dW.numel(), 0.0), (L.bias, db, db.numel(), 0.0)]
        upd += [(sh.w1, tb["dw1"], sh.d, model.reg_w), (sh.v, tb["dv"], sh.d * sh.kfm, model.reg_v),
                (sh.w0, tb["dw0"], 1, 0.0)]
        _lib.sgd_update_multi(upd, lr, st)
        sh.prepare()
        model.dnn._weights_changed()

    def bad_flag(self):
        """The device error flag's rs_flag bits (device tensor; resets):
        RS_FLAG_BAD_ID for an out-of-range id, RS_FLAG_LAYOUT for a table
        layout the dedup route cannot use."""
        v = self.err.clone()
        self.err.zero_()
        return v

    def clear_flags(self):
        """Restart the sticky id flag (a checked step reports its own ids)."""
        self.err.zero_()

    def check(self):
        raise_flag(self.bad_flag(), "sharded lookup")


class ShardedEmbeddingFM:
    """DeepFM embedding lookup + FM with the table row-sharded over a process
    group.  ``forward(dense[B,nd], ids[B,F]) -> logit[B,1]`` on every rank."""

    def __init__(self, vocab_sizes, k, nd, kfm, group=None, device=None, seed=0, ops=None, table_init=True,
                 world=None, rank=None):
        """world/rank: explicit partition without a process group (a rank of
        a simulated world in single-process tests); default: the group's."""
        self.group = group
        on = dist.is_initialized()
        self.world = int(world) if world is not None else (dist.get_world_size(group) if on else 1)
        self.rank = int(rank) if rank is not None else (dist.get_rank(group) if on else 0)
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        self.vocab_sizes = [int(v) for v in vocab_sizes]
        self.F, self.k, self.nd, self.kfm = len(self.vocab_sizes), int(k), int(nd), int(kfm)
        offs = [0]
        for v in self.vocab_sizes[:-1]:
            offs.append(offs[-1] + v)
        self.total_rows = sum(self.vocab_sizes)
        self.rows_per_rank = math.ceil(self.total_rows / self.world)
        lo = self.rank * self.rows_per_rank
        hi = min(self.total_rows, lo + self.rows_per_rank)
        self.row_range = (lo, hi)
        self.offsets = torch.tensor(offs, dtype=torch.int64, device=self.device)
        self.vocab = torch.tensor(self.vocab_sizes, dtype=torch.int64, device=self.device)
        nf = max(len(offs), 1)  # host copies (the fused kernels' kernel-argument metadata)
        self.host_offsets = (C.c_int64 * nf)(*offs[:len(self.vocab_sizes)])
        self.host_vocab = (C.c_int64 * nf)(*self.vocab_sizes)
        self.table_shard = torch.empty(max(hi - lo, 0), self.k, dtype=torch.float32, device=self.device)
        if table_init:
            g = torch.Generator(device=self.device)
            g.manual_seed(seed * 1009 + self.rank)
            self.table_shard.uniform_(-0.05, 0.05, generator=g)
        d = self.nd + self.F * self.k
        gen = torch.Generator(device="cpu")
        gen.manual_seed(seed)  # replicated dense parameters: same on every rank
        self.w0 = torch.zeros(1, device=self.device)
        self.w1 = (torch.randn(d, 1, generator=gen) * 0.05).to(self.device)
        self.v = (torch.randn(d, self.kfm, generator=gen) * 0.05).to(self.device)
        # partial protocol: owner o holds the contiguous field range its row
        # block intersects; messages are [B][slot_stride] local rows
        self.owner_field_ranges = []
        for o in range(self.world):
            lo_r, hi_r = o * self.rows_per_rank, min(self.total_rows, (o + 1) * self.rows_per_rank)
            cs = [c for c in range(self.F) if offs[c] < hi_r and offs[c] + self.vocab_sizes[c] > lo_r]
            self.owner_field_ranges.append((cs[0], len(cs)) if cs else (0, 0))
        self.slot_stride = max(1, max(n for _, n in self.owner_field_ranges))
        self.owner_fields = torch.tensor(self.owner_field_ranges, dtype=torch.int32, device=self.device)
        self.partial_width = (self.kfm + 2 + 3) // 4 * 4  # rs_fm_partial_width
        self.ops = ops if ops is not None else HipShardOps(self.device)
        self.prepared = None
        # world 1 skips the all-to-alls (a self-exchange is a copy); the bench
        # sets this to time the RCCL self-exchange as the N=1 point of its curve
        self._force_exchange = False
        if isinstance(self.ops, HipShardOps):
            self.prepare()

    def prepare(self):
        n = _lib.lib().rs_fm_prepared_size(self.nd, self.F, self.k, self.kfm)
        if self.prepared is None or self.prepared.numel() != n:
            self.prepared = torch.empty(n, dtype=torch.float32, device=self.device)
        call("rs_fm_prepare", ptr(self.w1), ptr(self.v), self.nd, self.F, self.k, self.kfm, ptr(self.prepared),
             _lib.stream())

    # -- the partial protocol (default forward)
    def _pbufs(self, B):
        pb = getattr(self, "_part_bufs", None)
        if pb is None or pb["B"] != B:
            W, S, P, dev = self.world, self.slot_stride, self.partial_width, self.device
            pb = {"B": B,
                  "send": torch.empty(W * B * S, dtype=torch.int32, device=dev),
                  "recv": torch.empty(W * B * S, dtype=torch.int32, device=dev),
                  "pout": torch.empty(W * B * P, dtype=torch.float32, device=dev),
                  "pin": torch.empty(W * B * P, dtype=torch.float32, device=dev)}
            self._part_bufs = pb
        return pb

    def forward(self, dense, ids, check=True, out=None):
        """FM logit [B,1] of the local batch (into ``out`` if given), partial
        protocol:
          1. rs_shard_field_route -> [world][B][S] local rows (-1 = not yours)
          2. all_to_all(rows ids)  -> what every requester asks of me  (RCCL)
          3. rs_shard_owner_fm     -> per (requester, sample) FM partials over
                                      my fields, [world][B][P] fp32
          4. all_to_all(partials)  -> every owner's partials of my samples (RCCL)
          5. rs_shard_fm_combine   -> sum owners in rank order + dense, logit
        Fixed, host-known message sizes (S*4 and P*4 bytes per sample and
        peer), no overflow case, no host sync unless ``check``."""
        B = ids.shape[0]
        pb = self._pbufs(B)
        if check:
            self.ops.clear_flags()  # a checked step reports its own ids only
        exchange = self.world > 1 or self._force_exchange
        send = self.ops.field_route(self, ids, pb["send"])
        recv = send
        if exchange:
            recv = pb["recv"]
            dist.all_to_all_single(recv, send, group=self.group)
        part = self.ops.owner_partials(self, recv, self.world * B, pb["pout"])
        if exchange:
            dist.all_to_all_single(pb["pin"], part, group=self.group)
            part = pb["pin"]
        logit = out if out is not None else torch.empty(B, 1, dtype=torch.float32, device=self.device)
        logit = self.ops.combine(self, part, dense, logit)
        if check:
            raise_flag(self.ops.bad_flag(), "sharded lookup", self.group, self.world)
        return logit

    # -- training: compile_fit's SGD on the FM logit, data parallel
    @property
    def d(self):
        return self.nd + self.F * self.k

    def _tbufs(self, B):
        tb = getattr(self, "_train_bufs", None)
        if tb is None or tb["B"] != B:
            W, dev, kfm, k = self.world, self.device, self.kfm, self.k
            lo, n_own = self.owner_field_ranges[self.rank]
            n_pairs = W * B
            tb = {"B": B,
                  "gs": torch.empty(B, kfm + 1, dtype=torch.float32, device=dev),
                  "gs_all": torch.empty(n_pairs, kfm + 1, dtype=torch.float32, device=dev),
                  "grad": torch.empty(self.d * (kfm + 1) + 1, dtype=torch.float32, device=dev),
                  "logit": torch.empty(B, 1, dtype=torch.float32, device=dev),
                  "xo": torch.empty(n_pairs, max(n_own, 1) * k, dtype=torch.float32, device=dev),
                  "drows": torch.empty(n_pairs, max(n_own, 1) * k, dtype=torch.float32, device=dev),
                  "zoff": torch.zeros(max(n_own, 1), dtype=torch.int64, device=dev),
                  "svocab": torch.full((max(n_own, 1),), self.table_shard.shape[0], dtype=torch.int64, device=dev),
                  "ws": torch.empty(max(_lib.lib().rs_embedding_sgd_workspace_size(n_pairs * max(n_own, 1))
                                        if isinstance(self.ops, HipShardOps) else 1, 1),
                                    dtype=torch.uint8, device=dev)}
            self._train_bufs = tb
        return tb

    def train_step(self, dense, ids, labels, lr=0.01, reg_w=1e-4, reg_v=1e-4, return_loss=False, check=True):
        """One SGD step of compile_fit (utils/compile_fit.py:9-15: SGD(lr),
        binary cross-entropy on sigmoid(FM logit), FMLayer's l2(reg_w) / l2(reg_v)
        on w1 / v — layer/interaction.py:94-104) over the GLOBAL batch (every
        rank's B samples; g scaled by 1 / (world * B)), as data-parallel
        training with the table row-sharded:
          forward  (the partial protocol, ``forward``) + rs_shard_fm_combine_grad
                   -> logit and each sample's [s | g] record
          all_gather([s | g])        -> every requester's records at every owner (RCCL)
          rs_fm_param_grads_strided  -> dense columns' dw1 / dv, dw0 (requester)
          rs_shard_owner_fm_grad     -> dL/drow of my owned lookups + my part of
                                        dw1 / dv over my fields' columns
          rs_embedding_sgd           -> row-sparse SGD of my shard (duplicates
                                        summed in global lookup order)
          all_reduce(dw1, dv, dw0)   -> replicated FM parameters stay identical (RCCL)
          rs_sgd_update_multi, rs_fm_prepare
        Every gradient comes from the pre-step weights.  Returns the per-sample
        losses of the local batch (before the step) if ``return_loss``."""
        B = ids.shape[0]
        W = self.world
        pb, tb = self._pbufs(B), self._tbufs(B)
        if check:
            self.ops.clear_flags()
        exchange = W > 1 or self._force_exchange
        send = self.ops.field_route(self, ids, pb["send"])
        recv = send
        if exchange:
            recv = pb["recv"]
            dist.all_to_all_single(recv, send, group=self.group)
        part = self.ops.owner_partials(self, recv, W * B, pb["pout"])
        if exchange:
            dist.all_to_all_single(pb["pin"], part, group=self.group)
            part = pb["pin"]
        loss = torch.empty(B, dtype=torch.float32, device=self.device) if return_loss else None
        self.ops.combine_grad(self, part, dense, labels, 1.0 / (W * B), tb["logit"], tb["gs"], loss)
        gs_all = tb["gs"]
        if exchange:
            gs_all = tb["gs_all"]
            dist.all_gather_into_tensor(gs_all, tb["gs"], group=self.group)
        grad = tb["grad"]
        grad.zero_()
        self.ops.dense_grads(self, dense, tb["gs"], grad)
        self.ops.owner_grads(self, recv, gs_all, grad, lr, tb)
        if W > 1:
            dist.all_reduce(grad, group=self.group)
        self.ops.apply(self, grad, lr, reg_w, reg_v)
        if check:
            raise_flag(self.ops.bad_flag(), "sharded lookup", self.group, W)
        return loss

    # -- the pipelined partial protocol: one all-to-all per batch
    def _sbufs(self, B):
        """Send/recv records of the pipelined stream."""
        sb = getattr(self, "_stream_bufs", None)
        if sb is None or sb["B"] != B:
            R = self.slot_stride + self.partial_width
            n = self.world * B * R
            sb = {"B": B, "R": R,
                  "send": torch.zeros(n, dtype=torch.int32, device=self.device),
                  "recv": torch.zeros(n, dtype=torch.int32, device=self.device)}
            self._stream_bufs = sb
        return sb

    def pipe_route(self, ids):
        """Prologue of a stream: the first batch's row-id words."""
        sb = self._sbufs(ids.shape[0])
        self.ops.field_route(self, ids, sb["send"], rec=sb["R"])

    @property
    def exchanges(self):
        """Whether steps run the all-to-alls (world 1 skips them unless the
        bench forces the RCCL self-exchange)."""
        return self.world > 1 or self._force_exchange

    # -- peer-mapped exchange (PeerExchange) in place of the RCCL all-to-all
    def use_peer_exchange(self, on=True, spin_limit=None):
        """Route the pipelined step's all-to-all (pipe_step / forward_stream)
        through PeerExchange mailboxes instead of RCCL.  Collective: every
        rank switches together (the mailboxes are created on first use, in
        the same order on every rank).  spin_limit: the mailboxes' bounded
        device waits (PeerExchange's default when None)."""
        self._peer_on = bool(on)
        if not hasattr(self, "_peers"):
            self._peers = {}
        if spin_limit is not None:
            self._peer_spin = int(spin_limit)

    def _peer(self, name, nbytes):
        ex = self._peers.get(name)
        if ex is None or ex.world * ex.block_bytes != nbytes:
            if ex is not None:
                ex.close()
            kw = {"spin_limit": self._peer_spin} if getattr(self, "_peer_spin", None) else {}
            ex = PeerExchange(nbytes // self.world, group=self.group, world=self.world, rank=self.rank,
                              device=self.device, **kw)
            self._peers[name] = ex
        return ex

    def close_peer_exchange(self):
        """Collective: unmap and free every mailbox (after the last step)."""
        for ex in getattr(self, "_peers", {}).values():
            ex.close()
        self._peers = {}
        self._peer_on = False

    def _peer_check(self):
        for ex in getattr(self, "_peers", {}).values():
            ex.check("sharded lookup (peer exchange)")

    def pipe_step(self, prev=None, cur=None, nxt=None):
        """One step of the pipelined partial protocol, for batch t = cur:
          all_to_all                  -> ONE collective: [row ids of t | partials of t-1]
          rs_shard_fm_pipe (1 launch) -> combine(t-1) into prev's out
                                         | owner partials of t  (ride the next exchange)
                                         | field route of t+1   (ditto)
        prev = (dense, out) of batch t-1, cur = ids of batch t (its row ids were
        routed by the previous step or pipe_route), nxt = (dense, ids) of
        batch t+1; any may be None."""
        B = next(x for x in (cur, prev and prev[0], nxt and nxt[1]) if x is not None).shape[0]
        sb = self._sbufs(B)
        if self.exchanges:
            if getattr(self, "_peer_on", False):
                # the records land in this rank's mailbox (valid until the next exchange)
                recv = self._peer("pipe", sb["send"].numel() * 4).all_to_all(sb["send"]).view(torch.int32)
            else:
                dist.all_to_all_single(sb["recv"], sb["send"], group=self.group)
                recv = sb["recv"]
            self.ops.pipe(self, recv, sb["send"], prev=prev, cur=cur, nxt=nxt)
        else:
            # no exchange: the launch must not write the records it reads, so
            # the two buffers alternate (read "send", write "recv", swap)
            self.ops.pipe(self, sb["send"], sb["recv"], prev=prev, cur=cur, nxt=nxt)
            sb["send"], sb["recv"] = sb["recv"], sb["send"]

    def forward_stream(self, batches, check=True):
        """FM logits of a sequence of local batches [(dense, ids), ...] with the
        pipelined partial protocol: batch t's row-id message and batch t-1's
        partials share one all-to-all and one launch, so a stream of n batches
        costs n + 1 collectives and n + 2 launches (vs 2n and 3n).  Every rank
        must pass the same number of batches.  Returns [logit [B,1] per batch]."""
        n = len(batches)
        outs = [torch.empty(ids.shape[0], 1, dtype=torch.float32, device=self.device) for _, ids in batches]
        if check:
            self.ops.clear_flags()
        if n:
            self.pipe_route(batches[0][1])
        for t in range(n + 1):
            prev = (batches[t - 1][0], outs[t - 1]) if t > 0 else None
            cur = batches[t][1] if t < n else None
            nxt = batches[t + 1] if t + 1 < n else None
            self.pipe_step(prev, cur, nxt)
        if check:
            raise_flag(self.ops.bad_flag(), "sharded lookup", self.group, self.world)
            if getattr(self, "_peer_on", False):
                self._peer_check()
        return outs

    # -- the TWO-DEEP pipelined partial protocol: the exchange off the critical path
    # Step t runs the exchange of batch t+1 BESIDE the pipe parts of batch t:
    #   E(t+1): [row ids of t+1 | partials of t-1]  (send slot (t+1) % 2 -> recv slot (t+1) % 2)
    #   P(t)  : combine(t-2) | owner partials of t | field route of t+2
    #           (reads recv slot t % 2, writes send slot t % 2)
    # E(t+1) needs only P(t-1)'s records and P(t) only E(t)'s, so the two
    # overlap: a step costs max(pipe, exchange) instead of pipe + exchange.
    # Peer exchange: ONE launch per step (rs_shard_fm_pipe_peer: the exchange
    # workgroups ride in the pipe launch; two-slot mailboxes).  RCCL: the
    # all-to-all stays on the caller's stream, the pipe launch goes to a side
    # stream; events order E(t+1) after P(t-1) and P(t) after E(t).  The
    # per-batch arithmetic is the one-deep step's, so the logits are
    # bit-identical to ``forward_stream``.
    def _s2bufs(self, B):
        sb = getattr(self, "_stream2_bufs", None)
        if sb is None or sb["B"] != B:
            R = self.slot_stride + self.partial_width
            n = self.world * B * R
            sb = {"B": B, "R": R, "n": n,
                  "send": torch.zeros(2, n, dtype=torch.int32, device=self.device),
                  "recv": torch.zeros(2, n, dtype=torch.int32, device=self.device)}
            self._stream2_bufs = sb
            self._p2_slot = 0
        return sb

    def _peer2(self, sb):
        """The two-slot mailboxes of the two-deep peer step (one PeerExchange
        of block 2 * B * R * 4 bytes: its data region is read as [2][world][B*R])."""
        blk = sb["B"] * sb["R"] * 4
        chunks = max(1, min(1024 // self.world, -(-blk // 16384)))
        ex = self._peers.get("pipe2")
        if ex is None or ex.block_bytes != 2 * blk:
            if ex is not None:
                ex.close()
            kw = {"spin_limit": self._peer_spin} if getattr(self, "_peer_spin", None) else {}
            ex = PeerExchange(2 * blk, group=self.group, world=self.world, rank=self.rank, device=self.device,
                              chunks=chunks, **kw)
            self._peers["pipe2"] = ex
        return ex

    def pipe2_prologue(self, ids0, ids1=None):
        """Prologue of a two-deep stream: route batches 0 and 1 into the send
        slots and run E(0) (launch t = -1).  Resets the slot parity."""
        sb = self._s2bufs(ids0.shape[0])
        self._p2_slot = 0
        self.ops.field_route(self, ids0, sb["send"][0], rec=sb["R"])
        if ids1 is not None:
            self.ops.field_route(self, ids1, sb["send"][1], rec=sb["R"])
        self._p2_slot = 1  # launch t = -1 has slot (-1) % 2 = 1: its exchange carries send slot 0
        self.pipe2_step(exchange=True, B=ids0.shape[0])

    def pipe2_step(self, prev=None, cur=None, nxt=None, exchange=True, B=None):
        """One two-deep step t (slot parity kept here, flipped every call):
        exchange E(t+1) of send slot (t+1) % 2 if ``exchange``, combine of
        prev = (dense, out) of batch t-2, owner partials of cur = ids of batch
        t, field route of nxt = ids of batch t+2 (any may be None)."""
        if B is None:
            B = next(x for x in (cur, prev and prev[0], nxt) if x is not None).shape[0]
        sb = self._s2bufs(B)
        if not self.exchanges:
            raise RuntimeError("pipe2_step: the two-deep step needs the exchange (world > 1 or a forced one)")
        slot = self._p2_slot
        xs = 1 - slot
        self._p2_slot = xs
        pipe = prev is not None or cur is not None or nxt is not None
        if getattr(self, "_peer_on", False):
            ex = self._peer2(sb)
            mbox = ex.recv.view(torch.int32).view(2, sb["n"])
            self.ops.pipe_peer(self, mbox[slot], sb["send"][slot], sb["send"][xs], xs, exchange, ex,
                               prev=prev, cur=cur, nxt=nxt, B=B)
            return
        on_gpu = self.device.type == "cuda"
        nx = (None, nxt) if nxt is not None else None  # ops.pipe takes (dense, ids)
        if exchange:
            if on_gpu and getattr(self, "_p2_evp", None) is not None:
                torch.cuda.current_stream(self.device).wait_event(self._p2_evp)
            dist.all_to_all_single(sb["recv"][xs], sb["send"][xs], group=self.group)
            if on_gpu:
                self._p2_eve_next = torch.cuda.Event()
                self._p2_eve_next.record(torch.cuda.current_stream(self.device))
        if pipe:
            if on_gpu:
                side = self._p2_side_stream()
                if getattr(self, "_p2_eve", None) is not None:
                    side.wait_event(self._p2_eve)
                with torch.cuda.stream(side):
                    self.ops.pipe(self, sb["recv"][slot], sb["send"][slot], prev=prev, cur=cur, nxt=nx)
                self._p2_evp = torch.cuda.Event()
                self._p2_evp.record(side)
            else:
                self.ops.pipe(self, sb["recv"][slot], sb["send"][slot], prev=prev, cur=cur, nxt=nx)
        if on_gpu:
            self._p2_eve = self._p2_eve_next if exchange else None

    def _p2_side_stream(self):
        s = getattr(self, "_p2_side", None)
        if s is None:
            s = self._p2_side = torch.cuda.Stream(self.device)
        return s

    def pipe2_begin(self):
        """Fork the side stream off the caller's stream and forget earlier
        events (the start of a captured / timed run of RCCL two-deep steps)."""
        self._p2_evp = self._p2_eve = None
        if self.device.type == "cuda" and not getattr(self, "_peer_on", False):
            self._p2_side_stream().wait_stream(torch.cuda.current_stream(self.device))

    def pipe2_join(self):
        """The caller's stream waits for the side stream's pipe launches (RCCL
        two-deep step; a no-op for the peer step, which has no side stream)."""
        if self.device.type == "cuda" and getattr(self, "_p2_side", None) is not None:
            torch.cuda.current_stream(self.device).wait_stream(self._p2_side)

    def forward_stream2(self, batches, check=True):
        """FM logits of a sequence of local batches [(dense, ids), ...] with the
        two-deep pipelined protocol (``pipe2_step``); bit-identical to
        ``forward_stream``.  n batches cost n + 3 launches (peer exchange: each
        carries the next batch's exchange) or n + 1 all-to-alls beside n + 2
        pipe launches (RCCL).  Every rank passes the same number of batches."""
        n = len(batches)
        outs = [torch.empty(ids.shape[0], 1, dtype=torch.float32, device=self.device) for _, ids in batches]
        if not n:
            return outs
        if check:
            self.ops.clear_flags()
        self._p2_evp = self._p2_eve = None
        self.pipe2_prologue(batches[0][1], batches[1][1] if n > 1 else None)
        for t in range(0, n + 2):
            exchange = t + 1 < n or 1 <= t <= n
            prev = (batches[t - 2][0], outs[t - 2]) if 0 <= t - 2 < n else None
            cur = batches[t][1] if t < n else None
            nxt = batches[t + 2][1] if t + 2 < n else None
            self.pipe2_step(prev, cur, nxt, exchange=exchange, B=batches[0][1].shape[0])
        self.pipe2_join()
        self._p2_evp = self._p2_eve = None
        if check:
            raise_flag(self.ops.bad_flag(), "sharded lookup", self.group, self.world)
            if getattr(self, "_peer_on", False):
                self._peer_check()
        return outs

    # -- the fixed-capacity row exchange (returns rows; forward_slots)
    def capacity(self, n):
        """Slots per (rank -> owner) message for n local lookups."""
        if self.world == 1:
            return max(n, 1)
        return min(n, ((int(math.ceil(1.15 * n / self.world)) + 64 + 63) // 64) * 64)

    def _bufs(self, B):
        bufs = getattr(self, "_slot_bufs", None)
        if bufs is None or bufs["B"] != B:
            n = B * self.F
            cap = self.capacity(n)
            W, dev = self.world, self.device
            bufs = {"B": B, "cap": cap,
                    "counts": torch.empty(W, dtype=torch.int32, device=dev),
                    "slot_of": torch.empty(n, dtype=torch.int32, device=dev),
                    "send": torch.full((W * cap,), -1, dtype=torch.int32, device=dev),  # -1 once (rs_capi.h)
                    "recv": torch.empty(W * cap, dtype=torch.int32, device=dev),
                    "reply": torch.empty(W * cap, self.k, dtype=torch.float32, device=dev),
                    "got": torch.empty(W * cap, self.k, dtype=torch.float32, device=dev),
                    "overflow": torch.zeros(1, dtype=torch.int32, device=dev),
                    "zoff": torch.zeros(self.F, dtype=torch.int64, device=dev),
                    "nslots": torch.full((self.F,), W * cap, dtype=torch.int64, device=dev)}
            self._slot_bufs = bufs
        return bufs

    def exchange_slots(self, ids):
        """Steps 1-4: returns (got [world*cap, k], slot_of [B*F]); the row of
        lookup j is got[slot_of[j]] (slot_of = -1: overflow / bad id)."""
        B = ids.shape[0]
        bufs = self._bufs(B)
        slot_of, send = self.ops.slot_bucketize(ids, self.offsets, self.vocab, self.rows_per_rank, self.world,
                                                bufs["cap"], bufs)
        exchange = self.world > 1 or self._force_exchange
        if not exchange:
            recv = send
        else:
            recv = bufs["recv"]
            dist.all_to_all_single(recv, send, group=self.group)
        reply = self.ops.gather_rows_into(self.table_shard, recv, bufs["reply"])
        if not exchange:
            got = reply
        else:
            got = bufs["got"]
            dist.all_to_all_single(got, reply, group=self.group)
        return got, slot_of

    # -- the exact exchange (fallback after an overflow, and the reference)
    def lookup(self, ids):
        """[B*F, k] embedding rows of the local batch in sample order."""
        counts, perm, send_rows = self.ops.bucketize(ids, self.offsets, self.vocab, self.rows_per_rank, self.world)
        if self.world == 1:
            reply = self.ops.gather_rows(self.table_shard, send_rows)
            return self.ops.unpermute(reply, perm)
        recv_counts = torch.empty_like(counts)
        dist.all_to_all_single(recv_counts, counts, group=self.group)
        splits = torch.stack([counts, recv_counts]).cpu().tolist()  # one host sync per step
        send_split, recv_split = splits[0], splits[1]
        recv_rows = torch.empty(sum(recv_split), dtype=torch.int32, device=self.device)
        dist.all_to_all_single(recv_rows, send_rows, recv_split, send_split, group=self.group)
        reply = self.ops.gather_rows(self.table_shard, recv_rows)
        got = torch.empty(sum(send_split), self.k, dtype=torch.float32, device=self.device)
        dist.all_to_all_single(got, reply, send_split, recv_split, group=self.group)
        return self.ops.unpermute(got, perm)

    def forward_exact(self, dense, ids):
        emb = self.lookup(ids)
        return self.ops.rows_fm(emb, dense, self.F, self.k, self.prepared, self.w0, self.kfm)

    def forward_slots(self, dense, ids, check=True, out=None):
        """FM logit [B,1] through the fixed-capacity ROW exchange (the rows of
        every lookup come back to the requester: EmbedLayer semantics).
        check=True: one host sync at the end of the step; a slot overflow is
        redone exactly, a bad id raises."""
        if check:
            self.ops.clear_flags()
        got, slot_of = self.exchange_slots(ids)
        bufs = self._bufs(ids.shape[0])
        logit = self.ops.slots_fm(got, slot_of, dense, self.F, self.k, self.prepared, self.w0, self.kfm, bufs,
                                  out=out)
        if check:
            # collective decision: every rank must take the same branch (the
            # exact fallback runs collectives; a lone raise would strand peers)
            f = self.ops.flags(bufs)
            if self.world > 1:
                dist.all_reduce(f, op=dist.ReduceOp.MAX, group=self.group)
            bad, overflow = f.tolist()
            if bad:
                raise_flag(torch.tensor([bad]), "sharded lookup")
            if overflow:
                return self.forward_exact(dense, ids)
        return logit

    __call__ = forward


def dropout_seed(seed, rank):
    """Seed of rank `rank`'s Dropout generator in ShardedDeepFM.train_step."""
    return ((int(seed) * 1000003 + 7919 * (int(rank) + 1)) * 2654435761) & (2 ** 64 - 1)


class ShardedDeepFM:
    """DeepFM (model/deepFM.py:15-31) with its embedding table row-sharded over
    a process group: BASELINE config 5.  ``forward(inputs) -> [B,1]``
    (post-sigmoid) on every rank for its local batch, where inputs is the
    reference's packed ``X[B, nd+F]`` or ``(dense[B,nd], ids[B,F])``.

    The DNN branch (``self.dnn(x)`` at model/deepFM.py:28-30) needs every
    row of x at the requester, so rows come back (EmbedLayer semantics,
    layer/core.py:273-280), over the same field-range records as the FM's
    partial protocol:
      1. rs_shard_row_route -> [world][B][S] local rows (-1 = not yours) and
                               slot_of[b*F + c] = where lookup (b, c)'s row
                               will land in the reply
      2. all_to_all(row ids)   (RCCL)
      3. rs_gather_rows       -> the owner serves [world*B*S, k] rows
      4. all_to_all(rows)      (RCCL)
      5. rs_deepfm_fwd        -> gather (from the exchange buffer, ids =
                               slot_of) + FM + DNN tower + sigmoid head, ONE
                               launch
    Fixed, host-known message sizes (no scan, no capacity, no overflow case),
    no host sync unless ``check``.  World 1 without a forced exchange runs
    step 5 on the table itself.  Dense parameters (FM w0 / w1 / v, the DNN)
    are replicated: every rank builds them from the same seed.  The local
    steps are pluggable (``ops``) so the protocol is testable over gloo on
    CPU (tests/test_sharded_gloo.py)."""

    def __init__(self, feature_columns, k, w_reg, v_reg, hidden_units, output_dim, activation, embed_dim=8,
                 group=None, device=None, seed=0, ops=None, table_init=True, world=None, rank=None, dedup=None):
        """dedup: None (field-range records) or the capacity fraction f in
        (0, 1] of the deduplicated exchange: each owner receives at most
        cap = f * B * slot_stride distinct rows per rank and step (rounded up
        to 64); f = 1 can never overflow, f < 1 moves fewer bytes when ids
        repeat (an overflow redoes the step without dedup when ``check``)."""
        from .layers import DNNLayer
        if dedup is not None and not (0.0 < float(dedup) <= 1.0):
            raise ValueError("dedup: a capacity fraction in (0, 1]")
        self.dedup = None if dedup is None else float(dedup)
        dense_cols, sparse_cols = feature_columns
        self.nd = len(dense_cols)
        vocabs = [int(f["feat_onehot_dim"]) for f in sparse_cols]
        self.reg_w, self.reg_v = float(w_reg), float(v_reg)
        self.emb = ShardedEmbeddingFM(vocabs, embed_dim, self.nd, k, group=group, device=device, seed=seed, ops=ops,
                                      table_init=table_init, world=world, rank=rank)
        sh = self.emb
        self.device, self.group, self.ops = sh.device, group, sh.ops
        self.world, self.rank, self.F, self.k, self.kfm = sh.world, sh.rank, sh.F, sh.k, sh.kfm
        self.dnn = DNNLayer(hidden_units, output_dim, activation, device=self.device, seed=seed * 7919 + 11)
        self.dnn.build(sh.d)
        self._in_rows = None
        self._seed = int(seed or 0)
        self._drop_rng = None
        # world 1: run the row protocol anyway (route, serve, finish; the
        # exchange is the identity) instead of the direct table path
        self.force_rows = False

    # -- parameters (replicated; Keras names of FMLayer + DNNLayer)
    @property
    def table_shard(self):
        return self.emb.table_shard

    def keras_weights(self):
        w = {"w0": self.emb.w0, "w1": self.emb.w1, "v": self.emb.v}
        w.update({f"dnn/{n}": p for n, p in self.dnn.keras_weights().items()})
        return w

    def fused_rows(self):
        """Tower input permutation: the fused kernel's LDS tile holds
        [emb F*k | dense nd], Keras rows are [dense nd | emb F*k]."""
        if self._in_rows is None:
            fk = self.F * self.k
            kp = (fk + self.nd + 15) // 16 * 16
            rows = torch.full((kp,), -1, dtype=torch.int32)
            rows[:fk] = torch.arange(fk, dtype=torch.int32) + self.nd
            rows[fk:fk + self.nd] = torch.arange(self.nd, dtype=torch.int32)
            self._in_rows = rows.to(self.device)
        return self._in_rows

    # -- the row exchange, step by step (forward = route, exchange, serve, exchange, finish)
    def _dedup_cap(self, B):
        full = B * self.emb.slot_stride
        return min((full + 63) // 64 * 64, max(64, (int(math.ceil(self.dedup * full)) + 63) // 64 * 64))

    def _rbufs(self, B, dedup=None):
        """Row-exchange buffers: field-range records (rec = slot_stride words
        per sample and owner) or, with dedup, cap distinct-row words per owner."""
        dedup = self.dedup is not None if dedup is None else dedup
        name = "_dedup_bufs" if dedup else "_row_bufs"
        rb = getattr(self, name, None)
        if rb is None or rb["B"] != B:
            W, S, dev, F = self.world, self.emb.slot_stride, self.device, self.F
            cap = self._dedup_cap(B) if dedup else B * S
            n = W * cap
            rb = {"B": B, "n": n, "dedup": dedup, "cap": cap, "rec": 1 if dedup else S,
                  "overflow": torch.zeros(1, dtype=torch.int32, device=dev),
                  "send": torch.empty(n, dtype=torch.int32, device=dev),
                  "recv": torch.empty(n, dtype=torch.int32, device=dev),
                  "slot_of": torch.empty(B, F, dtype=torch.int32, device=dev),
                  "reply": torch.empty(n, self.k, dtype=torch.float32, device=dev),
                  "got": torch.empty(n, self.k, dtype=torch.float32, device=dev),
                  # reverse exchange of the training step: dL/drow per slot
                  "gsend": torch.zeros(n, self.k, dtype=torch.float32, device=dev),
                  "grecv": torch.zeros(n, self.k, dtype=torch.float32, device=dev),
                  "zoff": torch.zeros(F, dtype=torch.int64, device=dev),
                  "nslots": torch.full((F,), n, dtype=torch.int64, device=dev)}
            if dedup and isinstance(self.ops, HipShardOps):
                rb["ws"] = torch.empty(max(_lib.lib().rs_shard_dedup_workspace_size(B * F, W), 1),
                                       dtype=torch.uint8, device=dev)
            setattr(self, name, rb)
        return rb

    def route(self, ids, rb):
        """Step 1: the row-id records (or distinct rows) to every owner and slot_of."""
        if rb["dedup"]:
            return self.ops.dedup_route(self.emb, ids, rb)
        return self.ops.row_route(self.emb, ids, rb["send"], rb["slot_of"])

    def _routed(self, ids, check):
        """Route the batch; with dedup and ``check``, a capacity overflow on
        any rank (collective decision: one host sync) reroutes it through the
        field-range records, so the step stays exact.  check=False with
        dedup < 1 is approximate: lookups past the capacity get slot -1, read
        a zero row (and set the sticky id flag) and drop their row gradient.
        Both flags restart here (device memsets, no sync), so an unchecked
        step never leaves a false IndexError or fallback to a checked one."""
        B = ids.shape[0]
        rb = self._rbufs(B)
        if rb["dedup"]:
            rb["overflow"].zero_()
        if check:
            self.ops.clear_flags()
        self.route(ids, rb)
        if rb["dedup"] and check:
            f = self.ops.overflow_flag(rb)
            if self.world > 1:
                dist.all_reduce(f, op=dist.ReduceOp.MAX, group=self.group)
            if bool(f.item()):
                rb = self._rbufs(B, dedup=False)
                self.route(ids, rb)
        return rb

    # -- pipelined forward: batch t+1's exchange beside batch t's fused kernel
    def _pipe_bufs(self, B, slot):
        """Row-exchange buffers of pipeline slot 0 / 1 (field-range records)."""
        key = f"_pipe_bufs{slot}"
        rb = getattr(self, key, None)
        if rb is None or rb["B"] != B:
            saved = getattr(self, "_row_bufs", None)
            self._row_bufs = None
            rb = self._rbufs(B, dedup=False)
            self._row_bufs = saved
            setattr(self, key, rb)
        return rb

    def exchange(self, ids, rb):
        """Steps 1-4 of forward into rb: route, all-to-all of the row ids, the
        owner's gather, all-to-all of the rows; rb["rows"] = the rows' buffer."""
        self.route(ids, rb)
        recv = rb["send"]
        if self.emb.exchanges:
            recv = rb["recv"]
            dist.all_to_all_single(recv, rb["send"], group=self.group)
        reply = got = self.serve(recv, rb["reply"])
        if self.emb.exchanges:
            got = rb["got"]
            dist.all_to_all_single(got, reply, group=self.group)
        rb["rows"] = got
        return rb

    def pipe_prologue(self, ids, slot=0):
        """Exchange of the first batch of a pipelined stream into `slot`."""
        return self.exchange(ids, self._pipe_bufs(ids.shape[0], slot))

    def pipe_step(self, cur, nxt=None, side=None):
        """One step of the pipelined forward (config 5, model/deepFM.py:23-31
        over the row-sharded table): rs_deepfm_fwd of batch t = cur = (dense,
        out, slot) from the rows its exchange left in `slot`, while batch
        t+1's exchange (nxt = (ids, slot'), route + two all-to-alls + the
        owner gather) runs into the other slot.  The collectives stay on the
        current stream and the kernel goes to a side stream that forks from
        and joins it every step (hub topology: RCCL collectives captured on a
        side stream crash hipGraph capture on this runtime, the capture
        stream's do not); the slot the exchange writes was last read by step
        t-1's kernel, which the previous join ordered before it.  Every rank
        must run the same steps (the collectives)."""
        dense, out, slot = cur
        if self.device.type != "cuda":  # CPU test doubles: the same steps, in order
            rb = self._pipe_bufs(dense.shape[0], slot)
            self.finish(dense, rb["rows"], rb, out)
            if nxt is not None:
                self.exchange(nxt[0], self._pipe_bufs(nxt[0].shape[0], nxt[1]))
            return out
        rb = self._pipe_bufs(dense.shape[0], slot)
        if nxt is None:
            self.finish(dense, rb["rows"], rb, out)
            return out
        main = torch.cuda.current_stream(self.device)
        side = side or self._side_stream()
        side.wait_stream(main)
        with torch.cuda.stream(side):
            self.finish(dense, rb["rows"], rb, out)
        ids_n, slot_n = nxt
        self.exchange(ids_n, self._pipe_bufs(ids_n.shape[0], slot_n))
        main.wait_stream(side)
        return out

    def _side_stream(self):
        if getattr(self, "_side", None) is None:
            self._side = torch.cuda.Stream(self.device)
        return self._side

    def forward_stream(self, batches, check=True):
        """DeepFM outputs of a sequence of local batches [(dense, ids), ...],
        pipelined: batch t+1's exchange overlaps batch t's fused kernel.
        Every rank must pass the same number of batches."""
        from .models import _split_criteo
        batches = [_split_criteo(b, self.nd, self.device) for b in batches]
        outs = [torch.empty(d.shape[0], 1, dtype=torch.float32, device=self.device) for d, _ in batches]
        if not batches:
            return outs
        if check:
            self.ops.clear_flags()  # an earlier unchecked step may have left the sticky flag set
        self.exchange(batches[0][1], self._pipe_bufs(batches[0][1].shape[0], 0))
        for t, (dense, _) in enumerate(batches):
            nxt = (batches[t + 1][1], (t + 1) % 2) if t + 1 < len(batches) else None
            self.pipe_step((dense, outs[t], t % 2), nxt)
        if check:
            raise_flag(self.ops.bad_flag(), "sharded DeepFM", self.group, self.world)
        return outs

    # -- peer-mapped exchange (PeerExchange) in place of the two RCCL all-to-alls
    def use_peer_exchange(self, on=True, spin_limit=None):
        """forward's exchanges through PeerExchange mailboxes: the row-id
        records (rs_peer_a2a), then the owner's rows gathered straight into
        the requesters' mailboxes (rs_peer_gather_a2a: rs_gather_rows and the
        row all-to-all become one launch).  Collective; k = 16 only."""
        if on and self.k != 16:
            raise ValueError("ShardedDeepFM.use_peer_exchange: k must be 16")
        self.emb.use_peer_exchange(on, spin_limit=spin_limit)

    def close_peer_exchange(self):
        self.emb.close_peer_exchange()

    def _peer_rows(self, rb):
        """Steps 2-4 over the mailboxes; None when this exchange cannot use
        them (record blocks not 16-B multiples)."""
        sh = self.emb
        n = rb["n"]
        nw = n // self.world
        if nw % 4 or not isinstance(self.ops, HipShardOps):
            return None
        recv = sh._peer("row_ids", n * 4).all_to_all(rb["send"]).view(torch.int32)
        got = sh._peer("rows", n * 64).gather_all_to_all(recv, nw, sh.table_shard, err=self.ops.err)
        return got.view(torch.float32).view(n, self.k)

    def serve(self, recv, reply):
        """Step 3 (owner): rows of the received record words (-1 -> zero row)."""
        return self.ops.gather_rows_into(self.emb.table_shard, recv, reply)

    def finish(self, dense, got, rb, out):
        """Step 5: the DeepFM forward from the exchange buffer."""
        return self.ops.deepfm_rows(self, got, rb, dense, out)

    # -- training: compile_fit's SGD step, data parallel, table row-sharded
    def _tbufs(self, B):
        tb = getattr(self, "_train_bufs", None)
        if tb is None or tb["B"] != B:
            sh, dev = self.emb, self.device
            W, S, k, d, kfm = self.world, sh.slot_stride, self.k, sh.d, sh.kfm
            layers = [(L, L.kernel.shape) for L in list(self.dnn.hidden_layer) + [self.dnn.output_layer]]
            sizes = [K * N + N for _, (K, N) in layers] + [d, d * kfm, 1]
            flat = torch.zeros(sum(sizes), dtype=torch.float32, device=dev)
            views, o = [], 0
            for _, (K, N) in layers:
                views.append((flat[o:o + K * N].view(K, N), flat[o + K * N:o + K * N + N]))
                o += K * N + N
            dw1, dv, dw0 = flat[o:o + d], flat[o + d:o + d + d * kfm].view(d, kfm), flat[o + d + d * kfm:]
            n_look = W * ((B * S + 63) // 64 * 64)  # either exchange layout
            tb = {"B": B, "flat": flat, "layers": layers, "dnn_views": views, "dw1": dw1, "dv": dv, "dw0": dw0,
                  "x": torch.empty(B, d, dtype=torch.float32, device=dev),
                  "fm": torch.empty(B, 1, dtype=torch.float32, device=dev),
                  "s": torch.empty(B, kfm, dtype=torch.float32, device=dev),
                  "g_fm": torch.empty(B, dtype=torch.float32, device=dev),
                  "g_dnn": torch.empty(B, dtype=torch.float32, device=dev),
                  "zoff": torch.zeros(S, dtype=torch.int64, device=dev),
                  "svocab": torch.full((S,), max(sh.table_shard.shape[0], 1), dtype=torch.int64, device=dev)}
            if isinstance(self.ops, HipShardOps):
                lib = _lib.lib()
                gmax = max(lib.rs_gemm_workspace_size(K, N, B) for _, (K, N) in layers)
                gmax = max(gmax, lib.rs_gemm_workspace_size(B, kfm, d))
                tb["gemm_ws"] = torch.empty(max(gmax, 1), dtype=torch.uint8, device=dev)
                tb["fm_prep"] = torch.empty(lib.rs_fm_prepared_size(d, 0, 0, kfm), dtype=torch.float32, device=dev)
                tb["emb_ws"] = torch.empty(max(lib.rs_embedding_sgd_workspace_size(n_look), 1), dtype=torch.uint8,
                                           device=dev)
            self._train_bufs = tb
        return tb

    def _dropout(self):
        """The rank's Dropout generator (rs_dropout): seeded from the model
        seed and the rank (dropout_seed), so ranks draw independent masks."""
        from .models import _Dropout
        if getattr(self, "_drop_rng", None) is None:
            self._drop_rng = _Dropout(dropout_seed(self._seed, self.rank), self.device)
        return self._drop_rng

    def _draws(self, B, rate):
        """(generator, rate, offsets): the next dropout draw of every hidden
        layer for a local batch of B (None at rate 0)."""
        if rate <= 0:
            return None
        rng, offs = self._dropout(), []
        for L in self.dnn.hidden_layer:
            offs.append(rng.take(B * L.units))
        return rng, rate, offs

    def train_step(self, inputs, labels, lr=0.01, return_loss=False, check=True, dropout=None):
        """One SGD step of compile_fit (utils/compile_fit.py:9-15: SGD(lr),
        binary cross-entropy on sigmoid(0.5 (FM + DNN)), FMLayer's l2
        regularisers; model/deepFM.py:23-31) over the GLOBAL batch — every
        rank's B samples, g scaled by 1/(world B) — as data-parallel training
        with the table row-sharded:
          forward exchange (rs_shard_row_route, all_to_all ids, owner
            rs_gather_rows, all_to_all rows)      -> every lookup's row here
          deepfm_grads  -> x, local forward + backward: this rank's share of
                           the DNN / FM gradients (flat buffer) and dL/dx
          rs_scatter_rows -> dL/drow into the row-exchange slot layout
          all_to_all(row gradients)  (RCCL; the reverse of the row exchange)
          owner: rs_embedding_sgd of the shard on the ids it served
          all_reduce(flat gradient)  (RCCL) -> rs_sgd_update_multi of the replicas
        Every gradient comes from the pre-step weights; every rank's update of
        the replicated parameters is identical.  DNNLayer's Dropout runs in
        training mode (rate = the layer's, dropout=False turns it off) with
        counter-based masks drawn per rank (_dropout).  Returns the per-sample
        losses of the local batch (before the step) if ``return_loss``."""
        from .models import _split_criteo, _dropout_rate
        from .layers import _to_device_f32
        sh = self.emb
        rate = _dropout_rate(self.dnn, dropout)
        if self.dnn.output_layer.units != 1 or any(l.activation not in (None, "linear", "relu")
                                                   for l in self.dnn.hidden_layer):
            raise NotImplementedError("ShardedDeepFM.train_step: output_dim 1, 'relu' / linear hidden layers")
        if isinstance(inputs, (tuple, list)) and not isinstance(self.ops, HipShardOps):
            dense, ids = inputs
            labels = torch.as_tensor(labels, dtype=torch.float32).reshape(-1)
        else:
            dense, ids = _split_criteo(inputs, self.nd, self.device)
            labels = _to_device_f32(labels, self.device).reshape(-1)
        B, W = ids.shape[0], self.world
        tb = self._tbufs(B)
        rb = self._routed(ids, check)
        recv = rb["send"]
        if sh.exchanges:
            recv = rb["recv"]
            dist.all_to_all_single(recv, rb["send"], group=self.group)
        reply = got = self.serve(recv, rb["reply"])
        if sh.exchanges:
            got = rb["got"]
            dist.all_to_all_single(got, reply, group=self.group)
        loss = torch.empty(B, dtype=torch.float32, device=self.device) if return_loss else None
        drop = self._draws(B, rate)  # this rank's draws: one offset range per hidden layer
        dx = self.ops.deepfm_grads(self, got, rb, dense, labels, 1.0 / (W * B), tb, loss, drop=drop)
        if rb["dedup"]:
            gsend = self.ops.dedup_grads(self, dx, rb)  # one row per distinct row
        else:
            gsend = self.ops.scatter_row_grads(self, dx, rb)
        grecv = gsend
        if sh.exchanges:
            grecv = rb["grecv"]
            dist.all_to_all_single(grecv, gsend, group=self.group)
        self.ops.owner_row_sgd(self, recv, grecv, lr, tb, rb["rec"])
        if W > 1:
            dist.all_reduce(tb["flat"], group=self.group)
        self.ops.deepfm_apply(self, tb, lr)
        if check:
            raise_flag(self.ops.bad_flag(), "sharded DeepFM", self.group, W)
        return loss

    def forward(self, inputs, check=True, out=None):
        from .models import _split_criteo
        sh = self.emb
        if isinstance(inputs, (tuple, list)) and not isinstance(self.ops, HipShardOps):
            dense, ids = inputs  # CPU test double: host tensors as given
        else:
            dense, ids = _split_criteo(inputs, self.nd, self.device)
        B = ids.shape[0]
        if out is None:
            out = torch.empty(B, 1, dtype=torch.float32, device=self.device)
        if check:
            self.ops.clear_flags()
        if not sh.exchanges and not self.force_rows and isinstance(self.ops, HipShardOps):
            self.ops.deepfm_table(self, ids, dense, out)  # world 1: the shard is the whole table
        else:
            rb = self._routed(ids, check)
            got = self._peer_rows(rb) if sh.exchanges and getattr(sh, "_peer_on", False) else None
            if got is None:
                recv = rb["send"]
                if sh.exchanges:
                    recv = rb["recv"]
                    dist.all_to_all_single(recv, rb["send"], group=self.group)
                reply = got = self.serve(recv, rb["reply"])
                if sh.exchanges:
                    got = rb["got"]
                    dist.all_to_all_single(got, reply, group=self.group)
            self.finish(dense, got, rb, out)
        if check:
            raise_flag(self.ops.bad_flag(), "sharded DeepFM", self.group, self.world)
            if getattr(sh, "_peer_on", False):
                sh._peer_check()
        return out

    __call__ = forward


def _deepfm_tower_args(model):
    dims = model.dnn._dims()
    n = len(dims) - 1
    acts = [_lib.ACT[l.activation] for l in model.dnn._layers()]
    return n, (C.c_int * (n + 1))(*dims), (C.c_int * n)(*acts)


def _deepfm_fused_ok(model):
    if not model.dnn.tower_ok() or model.dnn.output_layer.units != 1:
        return False
    n, dims, _ = _deepfm_tower_args(model)
    return bool(_lib.lib().rs_deepfm_fused_ok(model.nd, model.F, model.k, model.kfm, n, dims))


def _hip_deepfm(ops, model, ids, table, offs, vocab, dense, out, hmeta):
    """rs_deepfm_fwd_hm (one launch; hmeta = the (offsets, vocab) host arrays
    equal to offs / vocab) or, for shapes it does not take, the fused
    gather+FM kernel emitting x + the tower / per-layer DNN."""
    sh = model.emb
    if _deepfm_fused_ok(model):
        n, dims, acts = _deepfm_tower_args(model)
        mlp = model.dnn.prepared(model.fused_rows())
        call("rs_deepfm_fwd_hm", ptr(ids), _lib.id_kind(ids), ids.stride(0), ptr(dense), dense.stride(0), model.nd,
             ptr(table), ptr(offs), ptr(vocab), C.addressof(hmeta[0]), C.addressof(hmeta[1]), model.F, model.k,
             ptr(sh.prepared), ptr(sh.w0), model.kfm, n, dims, acts, ptr(mlp), 0.5, 0.5, ptr(out), None,
             ids.shape[0], ptr(ops.err), _lib.stream())
        return out
    from .layers import sigmoid_combine
    B = ids.shape[0]
    x = torch.empty(B, sh.d, dtype=torch.float32, device=model.device)
    fm = torch.empty(B, 1, dtype=torch.float32, device=model.device)
    call("rs_embed_fm_fwd", ptr(ids), _lib.id_kind(ids), ids.stride(0), ptr(dense), dense.stride(0), model.nd,
         ptr(table), ptr(offs), ptr(vocab), model.F, model.k, ptr(sh.prepared), ptr(sh.w0), model.kfm, ptr(fm),
         ptr(x), B, ptr(ops.err), _lib.stream())
    out.copy_(sigmoid_combine(fm, model.dnn(x), 0.5, 0.5))
    return out
