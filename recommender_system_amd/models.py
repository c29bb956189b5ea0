"""Keras-Model-compatible CTR models on the MI355X kernels.

Same names, constructor arguments and forward semantics as the reference's
models (Hcyand/recommender_system, algorithm/deep_learning/model/):

  FM(k, w_reg=1e-4, v_reg=1e-4)                                   model/fm.py:14-23
  DeepFM(feature_columns, k, w_reg, v_reg, hidden_units, output_dim, activation)
                                                                  model/deepFM.py:15-31
  DCN(feature_columns, hidden_units, output_dim, activation, layer_num, reg_w, reg_b)
                                                                  model/dcn.py:15-34
  PNN(feature_columns, mode, hidden_units, output_dim, activation='relu',
      dropout=0.2, use_fgcnn=False)                               model/pnn.py:14-53
  DIN(feature_columns, behavior_feature_list, att_hidden_units=(80, 40),
      dnn_hidden_units=(256, 128, 64), att_attention='prelu',
      dnn_activation='prelu', dnn_dropout=0.0)                    model/din.py:15-95
  NFM(feature_columns, hidden_units, output_dim, activation='relu', dropout=0)
                                                                  model/nfm.py:13-33
  AFM(feature_columns, mode)                                      model/afm.py:11-19
  FFM(feature_columns, k, w_reg=1e-4, v_reg=1e-4)                 model/ffm.py:10-22

Criteo-style models take the reference's packed input X[B, 13+F] (dense
features followed by label-encoded sparse ids, as floats — Keras casts them to
int32 inside Embedding, so ids are exact only below 2**24), or the pair
``(dense[B,13] float, ids[B,F] int32/int64)`` which lifts that limit.

Extra keyword ``embed_dim`` (default 8, the reference's EmbedLayer default)
sets the embedding width: the reference ignores feat['embed_dim'] and always
uses k=8 (layer/core.py:268-271), so 8 is the drop-in behaviour.

PNN runs with 3-D embeddings [B,F,k] (documented deviation: the reference's
rank-2 EmbedLayer makes PNN.call raise at model/pnn.py:38).  Modes 'inner',
'outer' and 'both' are built (forward and training); use_fgcnn=True is
outside this build's hot path and raises NotImplementedError; an unknown mode
raises the reference's ValueError.
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib
from ._lib import call, ptr
from .layers import (AFMLayer, Attention, BatchNormalization, CrossLayer, Dense, DNNLayer, EmbedLayer, FFMLayer,
                     FMLayer, InnerProductLayer, OuterProductLayer,
                     KerasModule, TowerMixin, sigmoid_combine, _ids_tensor, _to_device_f32, _ErrFlag)


def _split_criteo(inputs, nd, device):
    """(dense f32 [B,nd], ids [B,F]) from X[B,nd+F] or a (dense, ids) pair."""
    if isinstance(inputs, (tuple, list)):
        dense, ids = inputs
        return _to_device_f32(dense, device), _ids_tensor(ids, device)
    X = _to_device_f32(inputs, device)  # Keras autocast (float64 -> float32)
    return X[:, :nd], X[:, nd:]


def _subseed(gen):
    return int(torch.randint(0, 2 ** 31, (1,), generator=gen))


def _dnn_backward(layers, acts, delta, gw, emp, st, outs=None, drop=None):
    """Backward through Dense layers (relu or linear hidden activations):
    delta = dL/d(pre-activation) of the top layer; returns the (layer, dW, db)
    gradients and dL/d(acts[0]).  dW = a_in^T delta (split-K rs_gemm), db =
    column sums, delta_below = (delta W^T) [a_in > 0] (mask epilogue).
    outs: optional [(dW, db)] per layer to write into (contiguous views).
    drop: (_Dropout, rate, offsets) of the forward's hidden-layer dropout
    draws — delta_below is multiplied by the same keep / (1 - rate)."""
    B = acts[0].shape[0]
    grads = []
    for li in reversed(range(len(layers))):
        L, a_in = layers[li], acts[li]
        K_in, N_out = L.kernel.shape
        dW, db = outs[li] if outs is not None else (emp(K_in, N_out), emp(N_out))
        call("rs_gemm", 1, 0, K_in, N_out, B, 1.0, ptr(a_in), a_in.stride(0), ptr(delta), delta.stride(0), 0.0,
             ptr(dW), N_out, None, 0, *gw, st)
        call("rs_col_sum", ptr(delta), delta.stride(0), B, N_out, ptr(db), st)
        grads.append((L, dW, db))
        relu_below = li > 0 and layers[li - 1].activation == "relu"
        prev = emp(B, K_in)
        call("rs_gemm", 0, 1, B, K_in, N_out, 1.0, ptr(delta), delta.stride(0), ptr(L.kernel), N_out, 0.0,
             ptr(prev), K_in, ptr(a_in) if relu_below else None, a_in.stride(0), *gw, st)
        if drop is not None and 0 < li <= len(drop[2]):  # acts[li] is dropped hidden output li-1
            rng, rate, offs = drop
            rng.redraw(prev, rate, offs[li - 1], st)
        delta = prev
    if drop is not None:
        drop[0].end_step(st)
    return grads, delta


def _dnn_updates(grads, l2=0.0):
    """[(w, grad, n, l2)] of Dense layers' kernels and biases (for
    _lib.sgd_update_multi)."""
    out = []
    for L, dW, db in grads:
        out.extend([(L.kernel, dW, dW.numel(), l2), (L.bias, db, db.numel(), l2)])
    return out


def _dnn_apply(grads, lr, st, l2=0.0):
    _lib.sgd_update_multi(_dnn_updates(grads, l2), lr, st)


def _embedding_sgd(model, ids, dx, ldx, lr, st):
    """Row-sparse SGD of the looked-up rows from dL/dx's embedding block
    (columns nd.., row stride ldx): rs_embedding_sgd, duplicates summed in
    lookup order."""
    e = model.embed_layer
    B = ids.shape[0]
    ws_n = _lib.lib().rs_embedding_sgd_workspace_size(B * e.n_fields)
    ws = model.__dict__.get("_emb_ws")
    if ws is None or ws.numel() < ws_n:
        ws = model.__dict__["_emb_ws"] = torch.empty(ws_n, dtype=torch.uint8, device=model._dev)
    call("rs_embedding_sgd", ptr(e.table), e.total_rows, e.k, ptr(ids), _lib.id_kind(ids), ids.stride(0),
         ptr(e.field_offsets), ptr(e.field_vocab), e.n_fields, B, ptr(dx) + 4 * model.nd, ldx, float(lr), ptr(ws),
         None, st)


def _check_train_tower(name, dnn):
    if any(l.activation not in (None, "linear", "relu") for l in dnn.hidden_layer):
        raise NotImplementedError(f"{name}.train_step: 'relu' or linear hidden layers only")


class _Dropout:
    """DNNLayer's Dropout(rate) in training steps (layer/interaction.py:35,44;
    active under compile_fit's model.fit, utils/compile_fit.py:14): inverted
    dropout with counter-based masks (rs_dropout_at: Philox4x32-10, key =
    seed, one counter per 4 elements).  Every draw of a step takes the next
    offset range relative to a counter in DEVICE memory, the backward
    regenerates a draw's mask from the same (seed, counter + rel) instead of
    storing it, and end_step() advances the counter on the stream by the
    step's total — so a captured hipGraph of a training step draws fresh
    masks on every replay.  TF's own draws cannot be reproduced;
    oracle.dropout_multiplier restates this generator."""

    def __init__(self, seed, device=None):
        self.seed = int(seed) & (2 ** 64 - 1)
        self.base = torch.zeros(1, dtype=torch.int64, device=device if device is not None else "cuda")
        self.rel = 0

    @property
    def offset(self):
        """The absolute offset the next draw takes (reads the device counter)."""
        return int(self.base.item()) + self.rel

    def draw(self, t, rate, st):
        """Apply a fresh mask to t [rows, cols] in place; returns its offset
        relative to the step's counter."""
        off = self.rel
        self.redraw(t, rate, off, st)
        self.rel += (t.shape[0] * t.shape[1] + 3) // 4 * 4
        return off

    def take(self, n):
        """Reserve the next n elements' range (a draw made elsewhere)."""
        off = self.rel
        self.rel += (int(n) + 3) // 4 * 4
        return off

    def redraw(self, t, rate, rel, st):
        call("rs_dropout_at", ptr(t), t.stride(0), t.shape[0], t.shape[1], float(rate), self.seed, ptr(self.base),
             int(rel), st)

    def end_step(self, st):
        """Advance the device counter past this step's draws."""
        if self.rel:
            call("rs_dropout_advance", ptr(self.base), int(self.rel), st)
            self.rel = 0


def _dropout_rate(dnn, dropout):
    """The rate a training step applies: DNNLayer's own (Keras' fit runs the
    Dropout layers in training mode) unless dropout=False turns it off, or a
    float overrides it."""
    if dropout is False:
        return 0.0
    if dropout is None or dropout is True:
        return float(getattr(dnn, "dropout", 0) or 0)
    return float(dropout)


def _dropout_rng(model):
    rng = model.__dict__.get("_drop_rng")
    if rng is None:
        rng = model.__dict__["_drop_rng"] = _Dropout(_subseed(model._gen) * 2654435761 + 97, model._dev)
    return rng


def _dnn_train_forward(model, dnn, x, rate, st):
    """Hidden layers of DNNLayer in training: Dense + activation, then the
    dropout draw (rate > 0).  Returns (acts, drop) for _dnn_backward."""
    acts, offs = [x], []
    rng = _dropout_rng(model) if rate > 0 else None
    for layer in dnn.hidden_layer:
        a = layer(acts[-1])
        if rng is not None:
            offs.append(rng.draw(a, rate, st))
        acts.append(a)
    return acts, ((rng, rate, offs) if rng is not None else None)


def _gemm_ws(model, nbytes):
    ws = model.__dict__.get("_gemm_wsbuf")
    if ws is None or ws.numel() < max(nbytes, 1):
        ws = model.__dict__["_gemm_wsbuf"] = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=model._dev)
    return ws


class FM(KerasModule):
    """FM(k, w_reg, v_reg) — model/fm.py:14-23: sigmoid(FMLayer(x)).

    ``forward(x[B,n])`` takes the reference's one-hot matrix (any dense x).
    ``forward_onehot(dense, ids, field_offsets)`` takes its compact form and
    gathers rows of v/w1 instead of multiplying by zeros (same result: the
    one-hot block has exactly one 1 per field, utils/dataset.py:47-48)."""

    def __init__(self, k, w_reg=1e-4, v_reg=1e-4, device=None, seed=None, print_shape=False):
        super().__init__(device, seed)
        self.fm = FMLayer(k, w_reg, v_reg, device=device, seed=_subseed(self._gen))
        self.print_shape = print_shape  # the reference prints inputs.shape (model/fm.py:20)

    def forward(self, inputs):
        if self.print_shape:
            print(tuple(inputs.shape))
        logit = self.fm(inputs)
        return sigmoid_combine(logit)

    def forward_onehot(self, dense, ids, field_offsets, field_vocab, check_ids=True):
        dense = _to_device_f32(dense, self._dev)
        ids = _ids_tensor(ids, self._dev)
        offs = torch.as_tensor(field_offsets, dtype=torch.int64, device=self._dev)
        voc = torch.as_tensor(field_vocab, dtype=torch.int64, device=self._dev)
        B, nd = dense.shape
        n = nd + int(voc.sum())
        if not self.fm.built:
            self.fm.build(n)
        logit = torch.empty(B, 1, dtype=torch.float32, device=self._dev)
        err = _ErrFlag(self._dev)
        call("rs_fm_onehot_fwd", ptr(ids), _lib.id_kind(ids), ids.stride(0), ptr(dense), dense.stride(0), nd,
             ptr(offs), ptr(voc), ids.shape[1], ptr(self.fm.w1), ptr(self.fm.w0), ptr(self.fm.v), self.fm.k,
             ptr(logit), B, ptr(err.t), _lib.stream())
        if check_ids:
            err.check("FM")
        return sigmoid_combine(logit)

    def train_step(self, dense, ids, labels, field_offsets, field_vocab, lr=0.01, return_loss=False,
                   check_ids=True):
        """One step of compile_fit (utils/compile_fit.py:9-15: SGD(lr),
        binary cross-entropy, FMLayer's l2 regularisers) on a compact batch
        (dense [B,nd], label codes [B,F] of the one-hot x): one
        rs_fm_train_step call updates w0 / w1 / v in place.  Returns the
        per-sample losses before the step if ``return_loss``."""
        dense = _to_device_f32(dense, self._dev)
        ids = _ids_tensor(ids, self._dev)
        labels = _to_device_f32(labels, self._dev).reshape(-1)
        offs = torch.as_tensor(field_offsets, dtype=torch.int64, device=self._dev)
        voc = torch.as_tensor(field_vocab, dtype=torch.int64, device=self._dev)
        B, nd = dense.shape
        F = ids.shape[1]
        fm = self.fm
        if not fm.built:  # (a host sum: not inside a graph capture)
            fm.build(nd + int(voc.sum()))
        n = fm.w1.shape[0]
        ws_n = _lib.lib().rs_fm_train_workspace_size(B, F, fm.k, nd)
        ws = self.__dict__.get("_train_ws")
        if ws is None or ws.numel() < ws_n:
            ws = self.__dict__["_train_ws"] = torch.empty(ws_n, dtype=torch.uint8, device=self._dev)
        loss = torch.empty(B, dtype=torch.float32, device=self._dev) if return_loss else None
        err = _ErrFlag(self._dev)
        call("rs_fm_train_step", ptr(ids), _lib.id_kind(ids), ids.stride(0), ptr(dense), dense.stride(0), nd,
             ptr(offs), ptr(voc), F, fm.k, ptr(fm.w0), ptr(fm.w1), ptr(fm.v), n, ptr(labels), B, float(lr),
             float(fm.reg_w), float(fm.reg_b), ptr(ws), ptr(loss), ptr(err.t), _lib.stream())
        fm._invalidate()  # packed operand images of the old weights are stale
        if check_ids:
            err.check("FM.train_step")
        return loss


class DeepFM(KerasModule):
    """DeepFM — model/deepFM.py:15-31: x = [dense | EmbedLayer(sparse)],
    sigmoid(0.5*(FMLayer(x) + DNNLayer(x))).  Embedding lookup + concat + FM
    run as ONE fused kernel (rs_embed_fm_fwd) that also emits x for the DNN."""

    def __init__(self, feature_columns, k, w_reg, v_reg, hidden_units, output_dim, activation,
                 embed_dim=8, device=None, seed=None):
        super().__init__(device, seed)
        self.dense_feature_columns, self.sparse_feature_columns = feature_columns
        self.nd = len(self.dense_feature_columns)
        self.embed_layer = EmbedLayer(self.sparse_feature_columns, embed_dim, device=device, seed=_subseed(self._gen))
        d = self.nd + self.embed_layer.n_fields * embed_dim
        self.fm = FMLayer(k, w_reg, v_reg, device=device, seed=_subseed(self._gen), input_dim=d)
        self.dnn = DNNLayer(hidden_units, output_dim, activation, device=device, seed=_subseed(self._gen))
        self.dnn.build(d)
        self._err = _ErrFlag(self._dev)

    def fm_logit(self, inputs, x_out=None, check_ids=True):
        """The north-star hot path: ids -> rows -> FM logit in one launch."""
        dense, ids = _split_criteo(inputs, self.nd, self._dev)
        B = ids.shape[0]
        e = self.embed_layer
        prep = self.fm.prepared(self.nd, e.n_fields, e.k)
        logit = torch.empty(B, 1, dtype=torch.float32, device=self._dev)
        hoff, hvoc = e.host_meta()
        call("rs_embed_fm_fwd_hm", ptr(ids), _lib.id_kind(ids), ids.stride(0), ptr(dense), dense.stride(0), self.nd,
             ptr(e.table), ptr(e.field_offsets), ptr(e.field_vocab), hoff, hvoc, e.n_fields, e.k, ptr(prep),
             ptr(self.fm.w0), self.fm.k, ptr(logit), ptr(x_out), B, ptr(self._err.t), _lib.stream())
        if check_ids:
            self._err.check("DeepFM")
        return logit

    def fm_logit_stream(self, dense, ids, last_batch=None, min_blocks=1, out=None, check_ids=True):
        """The hot path over S consecutive batch requests in ONE launch
        (rs_embed_fm_fwd_hm_stream): dense [S, B, nd] f32, ids [S, B, F]
        int32 / int64 (contiguous per batch); the last batch may hold only
        ``last_batch`` samples.  Returns logits [S, B, 1] (rows past
        last_batch of the last batch untouched), each batch bit-identical to
        ``fm_logit`` on it alone."""
        S, B, F = ids.shape
        e = self.embed_layer
        if F != e.n_fields or dense.shape[:2] != (S, B) or dense.shape[2] != self.nd:
            raise ValueError("fm_logit_stream: dense [S, B, nd] and ids [S, B, F] expected")
        if ids.stride(2) != 1 or dense.stride(2) != 1:
            raise ValueError("fm_logit_stream: the last axis must be contiguous")
        prep = self.fm.prepared(self.nd, e.n_fields, e.k)
        logit = out if out is not None else torch.empty(S, B, 1, dtype=torch.float32, device=self._dev)
        hoff, hvoc = e.host_meta()
        call("rs_embed_fm_fwd_hm_stream", ptr(ids), _lib.id_kind(ids), ids.stride(1), ids.stride(0), ptr(dense),
             dense.stride(1), dense.stride(0), self.nd, ptr(e.table), hoff, hvoc, e.n_fields, e.k, ptr(prep),
             ptr(self.fm.w0), self.fm.k, ptr(logit), logit.stride(0), B, S, B if last_batch is None else last_batch,
             min_blocks, ptr(self._err.t), _lib.stream())
        if check_ids:
            self._err.check("DeepFM")
        return logit

    def train_step(self, inputs, labels, lr=0.01, return_loss=False, check_ids=True, dropout=None):
        """One step of compile_fit (utils/compile_fit.py:9-15: SGD(lr),
        binary cross-entropy on sigmoid(0.5 (FM + DNN)), FMLayer's l2
        regularisers) on a batch, every weight updated in place: the DNN's
        kernels/biases, w0 / w1 / v, and the looked-up embedding rows
        (row-sparse, duplicates summed in lookup order — rs_embedding_sgd).
        Forward with saved activations (rs_embed_gather, rs_dense_fwd,
        rs_fm_fwd), backward through rs_gemm / rs_col_sum / rs_fm_x_grad /
        rs_fm_param_grads, all gradients from the pre-step weights, then the
        updates.  Supports output_dim 1 and 'relu' / linear hidden layers.
        DNNLayer's Dropout runs in training mode as under Keras' fit (rate =
        the layer's, 0.2 by default; dropout=False turns it off): inverted
        dropout with counter-based masks (rs_dropout), the same masks in the
        backward."""
        dense, ids = _split_criteo(inputs, self.nd, self._dev)
        labels = _to_device_f32(labels, self._dev).reshape(-1)
        e, fm, dnn = self.embed_layer, self.fm, self.dnn
        layers = list(dnn.hidden_layer) + [dnn.output_layer]
        if dnn.output_layer.units != 1:
            raise NotImplementedError("DeepFM.train_step: output_dim 1 only")
        _check_train_tower("DeepFM", dnn)
        rate = _dropout_rate(dnn, dropout)
        B, dev, st = ids.shape[0], self._dev, _lib.stream()
        d, kfm = self.nd + e.n_fields * e.k, fm.k
        emp = lambda *shape: torch.empty(*shape, dtype=torch.float32, device=dev)
        # forward, keeping what the backward needs
        x = e.gather(ids, dense, check_ids=check_ids)
        acts, drop = _dnn_train_forward(self, dnn, x, rate, st)
        dnn_out = dnn.output_layer(acts[-1])
        fm_out = fm(x)
        s = emp(B, kfm)
        gws = self._gemm_ws(max(_lib.lib().rs_gemm_workspace_size(L.kernel.shape[0], L.kernel.shape[1], B)
                                for L in layers))
        gw = (ptr(gws), gws.numel())
        call("rs_gemm", 0, 0, B, kfm, d, 1.0, ptr(x), d, ptr(fm.v), kfm, 0.0, ptr(s), kfm, None, 0, *gw, st)
        g_fm, g_dnn = emp(B), emp(B)
        loss = emp(B) if return_loss else None
        call("rs_head_grad", ptr(fm_out), ptr(dnn_out), ptr(labels), B, 0.5, 0.5, ptr(g_fm), ptr(g_dnn), ptr(loss), st)
        grads, delta = _dnn_backward(layers, acts, g_dnn.view(B, 1), gw, emp, st, drop=drop)
        dx = delta  # [B, d]: the DNN's gradient w.r.t. x; the FM's is added next
        call("rs_fm_x_grad", ptr(x), d, ptr(s), ptr(fm.w1), ptr(fm.v), B, d, kfm, ptr(g_fm), ptr(dx), d, st)
        dw1, dv, dw0 = emp(d), emp(d, kfm), emp(1)
        call("rs_fm_param_grads", ptr(x), d, ptr(s), ptr(fm.v), B, d, kfm, ptr(g_fm), ptr(dw1), ptr(dv), ptr(dw0), st)
        # updates (every gradient above used the pre-step weights)
        _lib.sgd_update_multi(_dnn_updates(grads) + [(fm.w1, dw1, d, fm.reg_w), (fm.v, dv, d * kfm, fm.reg_b),
                                                     (fm.w0, dw0, 1, 0.0)], lr, st)
        _embedding_sgd(self, ids, dx, d, lr, st)
        self._weights_changed()  # packed operand images of the old weights are stale
        return loss

    def _gemm_ws(self, nbytes):
        return _gemm_ws(self, nbytes)

    def _fused_rows(self):
        """Tower input permutation for the fused kernel: its LDS tile holds
        [emb F*k | dense nd]; Keras rows are [dense nd | emb F*k]."""
        e = self.embed_layer
        fk = e.n_fields * e.k
        kp = (fk + self.nd + 15) // 16 * 16
        if getattr(self, "_in_rows", None) is None:
            rows = torch.full((kp,), -1, dtype=torch.int32)
            rows[:fk] = torch.arange(fk, dtype=torch.int32) + self.nd
            rows[fk:fk + self.nd] = torch.arange(self.nd, dtype=torch.int32)
            self._in_rows = rows.to(self._dev)
        return self._in_rows

    def fused_ok(self):
        e = self.embed_layer
        if not self.dnn.tower_ok():
            return False
        dims = self.dnn._dims()
        return bool(_lib.lib().rs_deepfm_fused_ok(self.nd, e.n_fields, e.k, self.fm.k, len(dims) - 1,
                                                   (C.c_int * len(dims))(*dims)))

    def forward_fused(self, inputs, check_ids=True, fm_logit=None):
        """DeepFM.call as ONE kernel (rs_deepfm_fwd)."""
        dense, ids = _split_criteo(inputs, self.nd, self._dev)
        B = ids.shape[0]
        e = self.embed_layer
        prep = self.fm.prepared(self.nd, e.n_fields, e.k)
        mlp = self.dnn.prepared(self._fused_rows())
        dims = self.dnn._dims()
        n = len(dims) - 1
        acts = [_lib.ACT[l.activation] for l in self.dnn._layers()]
        out = torch.empty(B, 1, dtype=torch.float32, device=self._dev)
        hoff, hvoc = e.host_meta()
        call("rs_deepfm_fwd_hm", ptr(ids), _lib.id_kind(ids), ids.stride(0), ptr(dense), dense.stride(0), self.nd,
             ptr(e.table), ptr(e.field_offsets), ptr(e.field_vocab), hoff, hvoc, e.n_fields, e.k, ptr(prep),
             ptr(self.fm.w0), self.fm.k, n, (C.c_int * (n + 1))(*dims), (C.c_int * n)(*acts), ptr(mlp), 0.5, 0.5,
             ptr(out), ptr(fm_logit), B, ptr(self._err.t), _lib.stream())
        if check_ids:
            self._err.check("DeepFM")
        return out

    def forward(self, inputs, check_ids=True):
        if self.fused_ok():
            return self.forward_fused(inputs, check_ids)
        return self.forward_unfused(inputs, check_ids)

    def forward_unfused(self, inputs, check_ids=True):
        """Fused gather+FM kernel emitting x, then the tower kernel."""
        dense, ids = _split_criteo(inputs, self.nd, self._dev)
        B = ids.shape[0]
        x = torch.empty(B, self.nd + self.embed_layer.n_fields * self.embed_layer.k, dtype=torch.float32,
                        device=self._dev)
        fm = self.fm_logit((dense, ids), x_out=x, check_ids=check_ids)
        if self.dnn.output_layer.units == 1 and self.dnn.tower_ok():
            # DNN tower + sigmoid(0.5*fm + 0.5*dnn) head in one launch
            return self.dnn.tower(x, extra=fm, c0=0.5, c1=0.5, head=True)
        dnn = self.dnn(x)
        return sigmoid_combine(fm, dnn, 0.5, 0.5)


class DCN(KerasModule):
    """DCN — model/dcn.py:15-34: sigmoid(Dense1([CrossLayer(x) | DNNLayer(x)]))."""

    def __init__(self, feature_columns, hidden_units, output_dim, activation, layer_num, reg_w=1e-4, reg_b=1e-4,
                 embed_dim=8, device=None, seed=None):
        super().__init__(device, seed)
        self.dense_feature_columns, self.sparse_feature_columns = feature_columns
        self.nd = len(self.dense_feature_columns)
        self.embed_layer = EmbedLayer(self.sparse_feature_columns, embed_dim, device=device, seed=_subseed(self._gen))
        d = self.nd + self.embed_layer.n_fields * embed_dim
        self.dense_layer = DNNLayer(hidden_units, output_dim, activation, device=device, seed=_subseed(self._gen))
        self.dense_layer.build(d)
        self.cross_layer = CrossLayer(layer_num, reg_w, reg_b, device=device, seed=_subseed(self._gen), input_dim=d)
        # Dense(1) followed by tf.nn.sigmoid (model/dcn.py:33): the sigmoid is
        # fused into the Dense epilogue; weights keep the Keras Dense names.
        self.output_layer = Dense(1, "sigmoid", device=device, seed=_subseed(self._gen), input_dim=d + output_dim)
        self.d = d
        self._err = _ErrFlag(self._dev)

    def cross_fused(self, inputs, out=None, check_ids=True):
        """CrossLayer([dense | EmbedLayer(ids)]) in ONE launch (rs_embed_cross_fwd):
        x0 is assembled in LDS and never written to HBM."""
        dense, ids = _split_criteo(inputs, self.nd, self._dev)
        B = ids.shape[0]
        e = self.embed_layer
        if out is None:
            out = torch.empty(B, self.d, dtype=torch.float32, device=self._dev)
        prep = self.cross_layer.prepared(self.d)
        hoff, hvoc = e.host_meta()  # field metadata also by value (the kernel-argument front end)
        call("rs_embed_cross_fwd_hm", ptr(ids), _lib.id_kind(ids), ids.stride(0), ptr(dense), dense.stride(0),
             self.nd, ptr(e.table), ptr(e.field_offsets), ptr(e.field_vocab), hoff, hvoc, e.n_fields, e.k,
             self.cross_layer.layer_num, ptr(prep), ptr(out), out.stride(0), B, ptr(self._err.t), _lib.stream())
        if check_ids:
            self._err.check("DCN")
        return out

    def _invalidate(self):
        self._fused_key = None

    def train_step(self, inputs, labels, lr=0.01, return_loss=False, check_ids=True, dropout=None):
        """One step of compile_fit on DCN (model/dcn.py:24-34, utils/compile_fit.py:
        9-15): SGD(lr), binary cross-entropy on sigmoid(Dense1([CrossLayer(x) |
        DNNLayer(x)])), CrossLayer's l2(reg_w) / l2(reg_b) regularisers
        (layer/interaction.py:57-73), every weight updated in place from the
        pre-step gradients.  The CrossNet runs as rs_cross_train_fwd (keeps
        x_1..x_L and x_l . w_l) and rs_cross_train_bwd (delta_l recursion);
        dw_l = x_l^T s_l and the Dense grads through rs_gemm, db_l / Dense
        biases through rs_col_sum, the looked-up rows by rs_embedding_sgd.
        DNNLayer's Dropout runs in training mode (counter-based masks,
        rs_dropout; dropout=False turns it off), as DeepFM.train_step."""
        dense, ids = _split_criteo(inputs, self.nd, self._dev)
        labels = _to_device_f32(labels, self._dev).reshape(-1)
        e, cl, dnn, out = self.embed_layer, self.cross_layer, self.dense_layer, self.output_layer
        rate = _dropout_rate(dnn, dropout)
        _check_train_tower("DCN", dnn)
        B, d, dev, st = ids.shape[0], self.d, self._dev, _lib.stream()
        od, Lc = dnn.output_layer.units, cl.layer_num
        dz_n = d + od
        emp = lambda *shape: torch.empty(*shape, dtype=torch.float32, device=dev)
        layers = list(dnn.hidden_layer) + [dnn.output_layer]
        gws = _gemm_ws(self, max(_lib.lib().rs_gemm_workspace_size(K, N, B)
                                 for K, N in [L.kernel.shape for L in layers] + [(d, 1), (dz_n, 1)]))
        gw = (ptr(gws), gws.numel())
        # forward, keeping what the backward needs
        x = e.gather(ids, dense, check_ids=check_ids)
        zc = emp(B, dz_n)  # [cross_out | dnn_out], the output Dense's input
        W = torch.stack([w.reshape(-1) for w in cl.cross_weight]).contiguous() if Lc else None
        Bc = torch.stack([b.reshape(-1) for b in cl.cross_bias]).contiguous() if Lc else None
        xs, gl = (emp(Lc, B, d), emp(Lc, B)) if Lc else (None, None)
        if Lc:
            call("rs_cross_train_fwd", ptr(x), d, d, Lc, ptr(W), ptr(Bc), B, ptr(xs), ptr(gl), ptr(zc), dz_n, st)
        else:
            zc[:, :d].copy_(x)
        acts, drop = _dnn_train_forward(self, dnn, x, rate, st)
        dnn.output_layer(acts[-1], out=zc[:, d:])
        logit = emp(B)
        call("rs_dense_fwd", ptr(zc), dz_n, ptr(out.kernel), ptr(out.bias), None, 0, ptr(logit), 1, B, dz_n, 1, st)
        g, g0 = emp(B), emp(B)
        loss = emp(B) if return_loss else None
        call("rs_head_grad", ptr(logit), ptr(logit), ptr(labels), B, 1.0, 0.0, ptr(g), ptr(g0), ptr(loss), st)
        # output Dense: dWo = zc^T g, dbo = sum g, dzc = g Wo^T
        dWo, dbo, dzc = emp(dz_n, 1), emp(1), emp(B, dz_n)
        call("rs_gemm", 1, 0, dz_n, 1, B, 1.0, ptr(zc), dz_n, ptr(g), 1, 0.0, ptr(dWo), 1, None, 0, *gw, st)
        call("rs_col_sum", ptr(g), 1, B, 1, ptr(dbo), st)
        call("rs_gemm", 0, 1, B, dz_n, 1, 1.0, ptr(g), 1, ptr(out.kernel), 1, 0.0, ptr(dzc), dz_n, None, 0, *gw, st)
        # DNN backward from dzc[:, d:], then the CrossNet's from dzc[:, :d]
        grads, dx = _dnn_backward(layers, acts, dzc[:, d:], gw, emp, st, drop=drop)
        if Lc:
            deltas, sl = emp(Lc, B, d), emp(Lc, B)
        else:
            deltas = sl = None
        call("rs_cross_train_bwd", ptr(x), d, d, Lc, ptr(W), B, ptr(gl), ptr(dzc), dz_n, ptr(deltas), ptr(sl),
             ptr(dx), d, st)
        dWc, dBc = emp(max(Lc, 1), d), emp(max(Lc, 1), d)
        for l in range(Lc):
            xl = x if l == 0 else xs[l - 1]
            call("rs_gemm", 1, 0, d, 1, B, 1.0, ptr(xl), d, ptr(sl[l]), 1, 0.0, ptr(dWc[l]), 1, None, 0, *gw, st)
            call("rs_col_sum", ptr(deltas[l]), d, B, d, ptr(dBc[l]), st)
        # updates
        upd = _dnn_updates(grads) + [(out.kernel, dWo, dz_n, 0.0), (out.bias, dbo, 1, 0.0)]
        for l in range(Lc):
            upd += [(cl.cross_weight[l], dWc[l], d, cl.reg_w), (cl.cross_bias[l], dBc[l], d, cl.reg_b)]
        _lib.sgd_update_multi(upd, lr, st)
        _embedding_sgd(self, ids, dx, d, lr, st)
        self.__dict__["_keep"] = (W, Bc)  # stream-ordered lifetime of the stacked operands
        self._weights_changed()
        return loss

    # ---- one-launch forward (rs_dcn_fwd)
    def _fused_layers(self):
        dl = self.dense_layer
        return list(dl.hidden_layer), dl.output_layer

    def fused_ok(self):
        hidden, last = self._fused_layers()
        if any(l.activation not in (None, "linear", "relu", "prelu", "sigmoid") for l in hidden):
            return False
        dims = [self.d] + [l.units for l in hidden] + [1]
        e = self.embed_layer
        return bool(_lib.lib().rs_dcn_fused_ok(self.nd, e.n_fields, e.k, self.cross_layer.layer_num, len(dims) - 1,
                                                (C.c_int * len(dims))(*dims)))

    def _fused_params(self):
        """Cross image over [w_0..w_{L-1}, w_o[:d]] and the DNN tower with its
        last layer folded with the output Dense's DNN half (cached)."""
        hidden, last = self._fused_layers()
        out = self.output_layer
        cl = self.cross_layer
        params = list(cl.cross_weight) + list(cl.cross_bias) + [out.kernel, out.bias, last.kernel, last.bias] + \
            [p for l in hidden for p in (l.kernel, l.bias, l.alpha) if p is not None]
        key = tuple((p._version, p.data_ptr()) for p in params)
        if getattr(self, "_fused_key", None) == key:
            return self._fused
        d = self.d
        with torch.no_grad():
            L = cl.layer_num
            W = torch.cat([w.reshape(1, d) for w in cl.cross_weight] + [out.kernel[:d].reshape(1, d)]).contiguous()
            Bb = torch.cat([b.reshape(1, d) for b in cl.cross_bias] + [torch.zeros(1, d, device=self._dev)]).contiguous()
            n = _lib.lib().rs_cross_prepared_size(d, L + 1)
            cross = torch.empty(n, dtype=torch.float32, device=self._dev)
            call("rs_cross_prepare", ptr(W), ptr(Bb), d, L + 1, ptr(cross), _lib.stream())
            # fold on rs_dense_fwd: wf = last.kernel @ wo2, bf = last.bias @ wo2 + out.bias
            wo2 = out.kernel[d:].reshape(-1, 1).contiguous()          # [out_dim, 1]
            h_last, od = last.kernel.shape
            kern = last.kernel.contiguous()
            wf = torch.empty(h_last, 1, dtype=torch.float32, device=self._dev)
            bf = torch.empty(1, dtype=torch.float32, device=self._dev)
            st = _lib.stream()
            call("rs_dense_fwd", ptr(kern), od, ptr(wo2), None, None, _lib.ACT[None], ptr(wf), 1, h_last, od, 1, st)
            call("rs_dense_fwd", ptr(last.bias), od, ptr(wo2), ptr(out.bias), None, _lib.ACT[None], ptr(bf), 1, 1, od, 1,
                 st)
            ks = [l.kernel for l in hidden] + [wf]
            bs = [l.bias for l in hidden] + [bf.contiguous()]
            als = [l.alpha for l in hidden] + [None]
            dims = [d] + [l.units for l in hidden] + [1]
            nl = len(ks)
            ci = (C.c_int * (nl + 1))(*dims)
            pa = lambda ts: (C.c_void_p * nl)(*[ptr(t) for t in ts])
            mlp = torch.empty(_lib.lib().rs_mlp_prepared_size(nl, ci), dtype=torch.float32, device=self._dev)
            call("rs_mlp_prepare", nl, ci, pa(ks), pa(bs), pa(als), None, ptr(mlp), _lib.stream())
            acts = [_lib.ACT[l.activation] for l in hidden] + [0]
        self._fused = (cross, mlp, dims, acts, (W, Bb, wf, bf))
        self._fused_key = key
        return self._fused

    def forward_fused(self, inputs, check_ids=True):
        """DCN.call as ONE kernel (rs_dcn_fwd)."""
        dense, ids = _split_criteo(inputs, self.nd, self._dev)
        B = ids.shape[0]
        e = self.embed_layer
        cross, mlp, dims, acts, _ = self._fused_params()
        n = len(dims) - 1
        out = torch.empty(B, 1, dtype=torch.float32, device=self._dev)
        hoff, hvoc = e.host_meta()
        call("rs_dcn_fwd_hm", ptr(ids), _lib.id_kind(ids), ids.stride(0), ptr(dense), dense.stride(0), self.nd,
             ptr(e.table), ptr(e.field_offsets), ptr(e.field_vocab), hoff, hvoc, e.n_fields, e.k,
             self.cross_layer.layer_num, ptr(cross), n, (C.c_int * (n + 1))(*dims), (C.c_int * n)(*acts), ptr(mlp),
             ptr(out), B, ptr(self._err.t), _lib.stream())
        if check_ids:
            self._err.check("DCN")
        return out

    def forward(self, inputs, check_ids=True):
        if self.fused_ok():
            return self.forward_fused(inputs, check_ids)
        return self.forward_unfused(inputs, check_ids)

    def forward_unfused(self, inputs, check_ids=True):
        dense, ids = _split_criteo(inputs, self.nd, self._dev)
        x = self.embed_layer.gather(ids, dense=dense, check_ids=check_ids)
        B = x.shape[0]
        z = torch.empty(B, self.d + self.dense_layer.output_layer.units, dtype=torch.float32, device=self._dev)
        self.cross_layer(x, out=z[:, :self.d])
        if self.dense_layer.tower_ok():
            self.dense_layer.tower(x, out=z[:, self.d:])
        else:
            h = x
            for layer in self.dense_layer.hidden_layer:
                h = layer(h)
            self.dense_layer.output_layer(h, out=z[:, self.d:])
        return self.output_layer(z)


class PNN(KerasModule):
    """PNN(feature_columns, mode, ...) — model/pnn.py:14-53, with 3-D
    embeddings (the reference reshapes them to 2-D before the product layers
    and crashes at :38).  mode 'inner' / 'outer' / 'both'; the DNN input
    [flat_emb | inner | outer] comes out of ONE launch (rs_embed_product_fwd).
    Returns the DNN logit (no sigmoid, as the reference)."""

    def __init__(self, feature_columns, mode, hidden_units, output_dim, activation="relu", dropout=0.2,
                 use_fgcnn=False, embed_dim=8, device=None, seed=None):
        super().__init__(device, seed)
        if mode not in ("inner", "outer", "both"):
            raise ValueError("Please choice mode's value in 'inner', 'outer', 'both'.")
        if use_fgcnn:
            raise NotImplementedError("PNN use_fgcnn=True: FGCNNLayer is outside this build's hot path")
        self.mode = mode
        self.dense_feature_columns, self.sparse_feature_columns = feature_columns
        self.nd = len(self.dense_feature_columns)
        self.embed_layer = EmbedLayer(self.sparse_feature_columns, embed_dim, device=device, seed=_subseed(self._gen))
        F = self.embed_layer.n_fields
        P = F * (F - 1) // 2
        self.inner_product_layer = InnerProductLayer(device=device)
        self.outer_product_layer = OuterProductLayer(device=device, seed=_subseed(self._gen))
        if mode != "inner":
            self.outer_product_layer.build(F, embed_dim)
        self.width = F * embed_dim + P * (2 if mode == "both" else 1)
        self.dnn_layer = DNNLayer(hidden_units, output_dim, activation, dropout, device=device,
                                  seed=_subseed(self._gen))
        self.dnn_layer.build(self.width)
        self._err = _ErrFlag(self._dev)

    def product_inputs(self, inputs, check_ids=True):
        """[flat_emb | inner | outer] (model/pnn.py:37-48) in one launch."""
        _, ids = _split_criteo(inputs, self.nd, self._dev)
        e = self.embed_layer
        B = ids.shape[0]
        out = torch.empty(B, self.width, dtype=torch.float32, device=self._dev)
        hoff, hvoc = e.host_meta()  # field metadata also by value (the kernel-argument front end)
        if self.mode == "inner":
            call("rs_embed_inner_fwd_hm", ptr(ids), _lib.id_kind(ids), ids.stride(0), ptr(e.table),
                 ptr(e.field_offsets), ptr(e.field_vocab), hoff, hvoc, e.n_fields, e.k, ptr(out), out.stride(0), B,
                 ptr(self._err.t), _lib.stream())
        else:
            call("rs_embed_product_fwd_hm", ptr(ids), _lib.id_kind(ids), ids.stride(0), ptr(e.table),
                 ptr(e.field_offsets), ptr(e.field_vocab), hoff, hvoc, e.n_fields, e.k,
                 1 if self.mode == "both" else 0, ptr(self.outer_product_layer.prepared()), ptr(out), out.stride(0),
                 B, ptr(self._err.t), _lib.stream())
        if check_ids:
            self._err.check("PNN")
        return out

    def forward(self, inputs, check_ids=True):
        return self.dnn_layer(self.product_inputs(inputs, check_ids))

    def train_step(self, inputs, labels, lr=0.01, return_loss=False, check_ids=True):
        """One step of the reference's own PNN loop (model/pnn.py:74-81:
        GradientTape, SGD(lr) over model.variables, loss
        tf.reduce_mean(losses.binary_crossentropy(y_train, pre)) on the DNN
        LOGIT — Keras' clipped probability form with the labels broadcast
        against the [B, 1] output, rs_bce_prob_grad), modes 'inner' /
        'outer' / 'both' (the loop's own example runs 'both', :61):
          [flat | inner | outer] in one launch (rs_embed_inner_fwd /
          rs_embed_product_fwd), DNN forward with saved activations
          (rs_dense_fwd), the DNN backward (split-K rs_gemm, rs_col_sum),
          rs_inner_product_bwd (dflat + sum_j dinner_ij e_j),
          rs_outer_product_bwd (+ sum g_p e_j W_p / e_i W_p^T) and
          rs_outer_product_w_grad (dW), then SGD of the DNN and of W and
          row-sparse rs_embedding_sgd of the tables.  The loop's loss has no
          regulariser (OuterProductLayer's l2 sits in model.losses, never
          added there).  The loop calls model(X) without training=True, so
          Dropout is the identity there too.  Returns the per-sample losses
          (before the step) if ``return_loss``."""
        dnn = self.dnn_layer
        if dnn.output_layer.units != 1:
            raise NotImplementedError("PNN.train_step: output_dim 1 only")
        _check_train_tower("PNN", dnn)
        _, ids = _split_criteo(inputs, self.nd, self._dev)
        labels = _to_device_f32(labels, self._dev).reshape(-1)
        e = self.embed_layer
        B, F, k, st = ids.shape[0], e.n_fields, e.k, _lib.stream()
        emp = lambda *shape: torch.empty(*shape, dtype=torch.float32, device=self._dev)
        x = self.product_inputs(inputs, check_ids)  # [B, F*k + P]: [flat | inner]
        layers = list(dnn.hidden_layer) + [dnn.output_layer]
        acts = [x]
        for layer in dnn.hidden_layer:
            acts.append(layer(acts[-1]))
        pre = dnn.output_layer(acts[-1])
        g = emp(B)
        loss = emp(B) if return_loss else None
        call("rs_bce_prob_grad", ptr(pre), pre.stride(0), ptr(labels), B, ptr(g), ptr(loss), st)
        gws = _gemm_ws(self, max(_lib.lib().rs_gemm_workspace_size(L.kernel.shape[0], L.kernel.shape[1], B)
                                 for L in layers))
        grads, delta = _dnn_backward(layers, acts, g.view(B, 1), (ptr(gws), gws.numel()), emp, st)
        w = self.width
        P = F * (F - 1) // 2
        de = emp(B, F * k)
        if self.mode in ("inner", "both"):
            call("rs_inner_product_bwd", ptr(x), w, ptr(delta) + 4 * F * k, w, ptr(delta), w, F, k, B, ptr(de),
                 F * k, st)
        else:
            de.copy_(delta[:, :F * k])
        dW = None
        if self.mode in ("outer", "both"):
            op = self.outer_product_layer
            o0 = F * k + (P if self.mode == "both" else 0)  # the outer block's first column
            dW = emp(*op.W.shape)
            call("rs_outer_product_bwd", ptr(x), w, ptr(delta) + 4 * o0, w, ptr(op.W), F, k, B, ptr(de), F * k, st)
            call("rs_outer_product_w_grad", ptr(x), w, ptr(delta) + 4 * o0, w, F, k, B, ptr(dW), st)
        upd = _dnn_updates(grads)
        if dW is not None:
            upd.append((self.outer_product_layer.W, dW, dW.numel(), 0.0))
        _lib.sgd_update_multi(upd, lr, st)
        ws_n = _lib.lib().rs_embedding_sgd_workspace_size(B * F)
        ws = self.__dict__.get("_emb_ws")
        if ws is None or ws.numel() < ws_n:
            ws = self.__dict__["_emb_ws"] = torch.empty(ws_n, dtype=torch.uint8, device=self._dev)
        call("rs_embedding_sgd", ptr(e.table), e.total_rows, k, ptr(ids), _lib.id_kind(ids), ids.stride(0),
             ptr(e.field_offsets), ptr(e.field_vocab), F, B, ptr(de), F * k, float(lr), ptr(ws), None, st)
        self._weights_changed()
        return loss


class DIN(TowerMixin, KerasModule):
    """DIN — model/din.py:15-95.  ``forward(inputs)`` takes the reference's
    dict: each dense / non-behaviour sparse feature [B,1] (or [B]), each
    behaviour feature [B,T] (0 = padding), and the candidate under the
    hard-coded key 'movie_id' (model/din.py:74) as [B, n_behaviour]: column i
    is the candidate's id for behaviour feature i (e.g. item id and category
    id, :73,77-79).  Behaviour features are taken in sparse-column order; their
    embeddings are concatenated along k and the mask comes from the first
    (:80)."""

    # train_step: the two-layer PReLU attention unit's forward and backward as
    # one launch each (rs_din_att_prelu_fwd / _bwd; False: the layer-by-layer
    # kernels; both are tested vs the oracle)
    fused_att_train = True

    def __init__(self, feature_columns, behavior_feature_list, att_hidden_units=(80, 40),
                 dnn_hidden_units=(256, 128, 64), att_attention="prelu", dnn_activation="prelu", dnn_dropout=0.0,
                 device=None, seed=None):
        super().__init__(device, seed)
        self.dense_feature_columns, self.sparse_feature_columns = feature_columns
        self.behavior_feature_list = list(behavior_feature_list)
        self.other_sparse = [f for f in self.sparse_feature_columns if f["feat"] not in self.behavior_feature_list]
        self.seq_feats = [f for f in self.sparse_feature_columns if f["feat"] in self.behavior_feature_list]
        if not self.seq_feats:
            raise ValueError("DIN: behavior_feature_list names no sparse feature column")
        self.other_sparse_num = len(self.other_sparse)
        self.dense_num = len(self.dense_feature_columns)
        self.behavior_num = len(self.behavior_feature_list)
        dev = device
        self.embed_sparse_layers = torch.nn.ModuleList(
            [EmbedLayer([f], k=f["embed_dim"], device=dev, seed=_subseed(self._gen)) for f in self.other_sparse])
        self.embed_seq_layers = torch.nn.ModuleList(
            [EmbedLayer([f], k=f["embed_dim"], device=dev, seed=_subseed(self._gen)) for f in self.seq_feats])
        self.att_layer = Attention(att_hidden_units, att_attention, device=dev, seed=_subseed(self._gen))
        self.bn_layer = BatchNormalization(device=dev)
        act = "prelu" if dnn_activation == "prelu" else "dice"
        self.dense_layer = torch.nn.ModuleList(
            [Dense(u, activation=act, device=dev, seed=_subseed(self._gen)) for u in dnn_hidden_units])
        self.dropout = dnn_dropout
        self.out_layer = Dense(1, activation="sigmoid", device=dev, seed=_subseed(self._gen))
        self._err = _ErrFlag(self._dev)

    def _behaviour_embed(self, ids_cols, rows, check_ids):
        """[rows, K] = concat_i embed_seq_layers[i](ids_cols[i]) along k."""
        K = sum(l.k for l in self.embed_seq_layers)
        out = torch.empty(rows, K, dtype=torch.float32, device=self._dev)
        col = 0
        for ids, layer in zip(ids_cols, self.embed_seq_layers):
            layer.gather(ids, out=out[:, col:col + layer.k], check_ids=check_ids)
            col += layer.k
        return out

    def forward(self, inputs, check_ids=True):
        dev = self._dev
        nb = len(self.seq_feats)
        hists = [_ids_tensor(inputs[f["feat"]], dev) for f in self.seq_feats]
        B, T = hists[0].shape
        if any(h.shape != (B, T) for h in hists):
            raise ValueError("DIN: every behaviour feature must be [B, T]")
        cand = _ids_tensor(inputs["movie_id"], dev).reshape(B, -1)
        if cand.shape[1] != nb:
            raise ValueError(f"DIN: inputs['movie_id'] needs one candidate id per behaviour feature ({nb})")
        K = sum(l.k for l in self.embed_seq_layers)
        other_k = sum(l.k for l in self.embed_sparse_layers)
        width = 2 * K + other_k + self.dense_num
        emb = torch.empty(B, width, dtype=torch.float32, device=dev)
        if self.att_layer.out_kernel is None:
            self.att_layer.build(T, K)
        if nb == 1 and self.att_layer.ids_ok(K) and self.fused_call:
            y = self._forward_one_launch(inputs, hists[0], cand, K, width, check_ids)
            if y is not None:
                return y
        if nb == 1 and self.att_layer.ids_ok(K):
            # keys/values read through the ids from the (L2-resident) table; the
            # pooled rows and the candidate rows go straight into emb, in the
            # attention's one launch (rs_din_attention_ids_cand_fwd)
            seq_layer = self.embed_seq_layers[0]
            self.att_layer.forward_ids(seq_layer.table, int(seq_layer.vocab_sizes[0]), hists[0], cand,
                                       err=self._err.t, out=emb[:, :K], cand_out=emb[:, K:2 * K])
            if check_ids:
                self._err.check("DIN")
        else:
            item_embed = self._behaviour_embed([cand[:, i:i + 1] for i in range(nb)], B, check_ids)
            seq_embed = self._behaviour_embed([h.reshape(B * T, 1) for h in hists], B * T, check_ids)
            seq_embed = seq_embed.view(B, T, K)
            mask = (hists[0] != 0).to(torch.float32)  # model/din.py:80: the first behaviour feature
            att_emb = self.att_layer([item_embed, seq_embed, seq_embed, mask])
            emb[:, K:2 * K] = item_embed
            emb[:, :K] = att_emb
        if self.out_layer.kernel is not None and self.tower_ok():
            # BatchNormalization + PReLU MLP + Dense(1, sigmoid) in one launch,
            # the other sparse embeddings and the dense features read
            # straight into its input tile (no concat launch, no buffer)
            if self.bn_layer.gamma is None:
                self.bn_layer.build(emb.shape[-1])
            pieces = self._rest_pieces(inputs, 2 * K, B)
            if self.pieces_in_tower and 0 < len(pieces) <= 16 and width <= 64:
                y = self._tower_pieces(emb, pieces, self.bn_layer.affine())
                if check_ids:
                    self._err.check("DIN")
                return y
            self._concat_rest(inputs, emb, 2 * K, B, check_ids)
            return self.tower(emb, in_affine=self.bn_layer.affine())
        self._concat_rest(inputs, emb, 2 * K, B, check_ids)
        x = self.bn_layer(emb)
        for layer in self.dense_layer:
            x = layer(x)
        return self.out_layer(x)

    # DIN.call from the ids to the logit as ONE launch (rs_din_forward_ids:
    # the attention unit, then bn + the PReLU tower + Dense(1, sigmoid) in the
    # same workgroups; bit-identical to the two launches below, which stay the
    # path for shapes it does not take and for fused_call = False)
    fused_call = True

    def _forward_one_launch(self, inputs, hist, cand, K, width, check_ids):
        if self.out_layer.kernel is None or not self.tower_ok() or not self.pieces_in_tower or width > 64:
            return None
        B, T = hist.shape
        pieces = self._rest_pieces(inputs, 2 * K, B)
        if not 0 < len(pieces) <= 16:
            return None
        att = self.att_layer
        if att.out_kernel is None:
            att.build(T, K)
        h1, h2 = att.hidden_units
        ls = self._layers()
        n = len(ls)
        dims = self._dims()
        cdims = (C.c_int * (n + 1))(*dims)
        if T != att.T or not _lib.lib().rs_din_forward_ids_supported(T, K, h1, h2, n, cdims):
            return None
        if self.bn_layer.gamma is None:
            self.bn_layer.build(width)
        sc, sh = self.bn_layer.affine()
        seq_layer = self.embed_seq_layers[0]
        y = torch.empty(B, 1, dtype=torch.float32, device=self._dev)
        k = len(pieces)
        arr = lambda ctype, vals: (ctype * k)(*vals)
        call("rs_din_forward_ids", ptr(hist), _lib.id_kind(hist), hist.stride(0), ptr(cand), cand.stride(0), T, K,
             ptr(seq_layer.table), int(seq_layer.vocab_sizes[0]), h1, h2, ptr(att.prepared_ids(K)), None, 0,
             ptr(sc), ptr(sh), n, cdims, (C.c_int * n)(*[_lib.ACT[l.activation] for l in ls]),
             ptr(self.prepared()), ptr(y), y.stride(0), k, arr(C.c_int, [p[0] for p in pieces]),
             arr(C.c_int, [p[1] for p in pieces]), arr(C.c_int, [p[2] for p in pieces]),
             arr(C.c_void_p, [ptr(p[3]) for p in pieces]), arr(C.c_int64, [p[3].stride(0) for p in pieces]),
             arr(C.c_void_p, [ptr(p[4]) if p[4] is not None else None for p in pieces]),
             arr(C.c_int64, [p[5] for p in pieces]), B, ptr(self._err.t), _lib.stream())
        if check_ids:
            self._err.check("DIN")
        return y

    # DIN.call's tower reads the other sparse embeddings and the dense
    # features itself (rs_mlp_affine_pieces_fwd); False: one rs_concat_pieces
    # launch writes them into the concat first (both tested)
    pieces_in_tower = True

    def _rest_pieces(self, inputs, col, B):
        """(width, column, kind, source, table, vocab) of the other sparse
        embeddings and the dense features, from column `col` on
        (model/din.py:64-69,84-85)."""
        dev = self._dev
        pieces = []
        for f, layer in zip(self.other_sparse, self.embed_sparse_layers):
            ids = _ids_tensor(inputs[f["feat"]], dev).reshape(B, 1)
            pieces.append((layer.k, col, _lib.id_kind(ids), ids, layer.table, int(layer.vocab_sizes[0])))
            col += layer.k
        for f in self.dense_feature_columns:
            x = _to_device_f32(inputs[f["feat"]], dev).reshape(B, 1)
            pieces.append((1, col, -1, x, None, 0))
            col += 1
        return pieces

    def _tower_pieces(self, emb, pieces, affine):
        """BN + PReLU MLP + head over [emb[:, :2K] | pieces] in one launch."""
        ls = self._layers()
        n = len(ls)
        dims = self._dims()
        B = emb.shape[0]
        out = torch.empty(B, dims[-1], dtype=torch.float32, device=self._dev)
        sc, sh = affine
        k = len(pieces)
        arr = lambda ctype, vals: (ctype * k)(*vals)
        call("rs_mlp_affine_pieces_fwd", ptr(emb), emb.stride(0), ptr(sc), ptr(sh), n, (C.c_int * (n + 1))(*dims),
             (C.c_int * n)(*[_lib.ACT[l.activation] for l in ls]), ptr(self.prepared()), ptr(out), out.stride(0), 0,
             None, 1.0, 1.0, B, k, arr(C.c_int, [p[0] for p in pieces]), arr(C.c_int, [p[1] for p in pieces]),
             arr(C.c_int, [p[2] for p in pieces]), arr(C.c_void_p, [ptr(p[3]) for p in pieces]),
             arr(C.c_int64, [p[3].stride(0) for p in pieces]),
             arr(C.c_void_p, [ptr(p[4]) if p[4] is not None else None for p in pieces]),
             arr(C.c_int64, [p[5] for p in pieces]), ptr(self._err.t), _lib.stream())
        return out

    def _concat_rest(self, inputs, emb, col, B, check_ids):
        """The other sparse embeddings and the dense features into emb[:, col:]
        (model/din.py:64-69,84-85): ONE rs_concat_pieces launch for up to 16
        pieces, one launch per piece beyond."""
        pieces = self._rest_pieces(inputs, col, B)
        for i in range(0, len(pieces), 16):
            part = pieces[i:i + 16]
            n = len(part)
            arr = lambda ctype, vals: (ctype * n)(*vals)
            call("rs_concat_pieces", n, arr(C.c_int, [p[0] for p in part]), arr(C.c_int, [p[1] for p in part]),
                 arr(C.c_int, [p[2] for p in part]), arr(C.c_void_p, [ptr(p[3]) for p in part]),
                 arr(C.c_int64, [p[3].stride(0) for p in part]),
                 arr(C.c_void_p, [ptr(p[4]) if p[4] is not None else None for p in part]),
                 arr(C.c_int64, [p[5] for p in part]), ptr(emb), emb.stride(0), B, ptr(self._err.t), _lib.stream())
        if check_ids and pieces:
            self._err.check("DIN")

    def _layers(self):
        return list(self.dense_layer) + [self.out_layer]

    def train_step(self, inputs, labels, lr=0.01, return_loss=False, check_ids=True, dropout=None):
        """One step of compile_fit on DIN (utils/compile_fit.py:9-15: Keras
        fit, SGD(lr), binary_crossentropy on the sigmoid output — Keras takes
        the sigmoid's logit) with DIN.call in training mode (model/din.py:
        56-95): BatchNormalization normalises with the batch's own mean and
        biased variance and moves its averages (momentum 0.99), and so do
        the Dice layers' BatchNormalizations (att_attention / dnn_activation
        'prelu' — the reference defaults — or 'dice': rs_dice_train_fwd/_bwd).
          forward: behaviour / candidate rows (rs_embed_gather), the
          attention input [q, k, q-k, q*k] (rs_din_att_concat), each
          attention Dense (rs_dense_fwd) + PReLU over [T, h] alphas
          (rs_prelu_rows_fwd, kept pre-activations), the score Dense, masked
          softmax + pool (rs_masked_softmax_pool), rs_bn_train_fwd, the PReLU
          DNN and the output logit;
          backward: rs_head_grad, per Dense layer split-K rs_gemm / rs_col_sum
          / rs_prelu_rows_bwd, rs_bn_train_bwd, rs_masked_softmax_pool_bwd,
          rs_din_att_concat_bwd; then one rs_sgd_update_multi over every dense parameter
          and row-sparse rs_embedding_sgd of the behaviour tables (history
          rows, then candidates) and the other sparse tables.
        Dropout(dnn_dropout) after the DNN (:93) runs in training mode: one
        rs_dropout draw on the last DNN output, the same mask regenerated on
        its gradient (dropout=False turns it off, a float overrides the
        rate).  Returns per-sample losses (before the step) if
        ``return_loss``."""
        att, bn = self.att_layer, self.bn_layer
        rate = _dropout_rate(self, dropout)
        dev, st = self._dev, _lib.stream()
        nb = len(self.seq_feats)
        hists = [_ids_tensor(inputs[f["feat"]], dev) for f in self.seq_feats]
        B, T = hists[0].shape
        if any(h.shape != (B, T) for h in hists):
            raise ValueError("DIN: every behaviour feature must be [B, T]")
        cand = _ids_tensor(inputs["movie_id"], dev).reshape(B, -1)
        if cand.shape[1] != nb:
            raise ValueError(f"DIN: inputs['movie_id'] needs one candidate id per behaviour feature ({nb})")
        if self.out_layer.kernel is None:
            self.forward(inputs, check_ids)  # Keras build on the first call
        if T != att.T:
            raise ValueError(f"Attention built for T={att.T} (PReLU alpha is [T,h]); got T={T}")
        labels = _to_device_f32(labels, dev).reshape(-1)
        emp = lambda *shape: torch.empty(*shape, dtype=torch.float32, device=dev)
        K = sum(l.k for l in self.embed_seq_layers)
        M = B * T
        width = 2 * K + sum(l.k for l in self.embed_sparse_layers) + self.dense_num
        shapes = [(W.shape[0], W.shape[1], M) for W in att.kernels] + [(att.out_kernel.shape[0], 1, M)]
        shapes += [(L.kernel.shape[0], L.kernel.shape[1], B) for L in self._layers()]
        lb = _lib.lib()
        # one scratch buffer for every stream-ordered call below (gemm split-K
        # slices, column-sum slices, the PReLU backward's products)
        need = [max(lb.rs_gemm_workspace_size(kin, n, m), lb.rs_gemm_workspace_size(m, kin, n),
                    lb.rs_col_sum_workspace_size(m, n)) for kin, n, m in shapes]
        need += [lb.rs_prelu_rows_bwd_workspace_size(M, W.shape[1], T) for W in att.kernels]
        need += [lb.rs_prelu_rows_bwd_workspace_size(B, L.units, 1) for L in self.dense_layer]
        need += [lb.rs_dice_train_workspace_size(M, 4 * K)] if att.activation == "dice" else []
        need += [lb.rs_dice_train_workspace_size(B, L.units) for L in self.dense_layer if L.activation == "dice"]
        # the PReLU unit with two hidden layers (the reference default (80, 40)):
        # rs_din_att_prelu_bwd when its shape fits; otherwise layer by layer
        att_fused = (self.fused_att_train and att.activation == "prelu" and len(att.kernels) == 2
                     and lb.rs_din_att_prelu_bwd_workspace_size(B, T, 4 * K, *att.kernels[1].shape) >= 0)
        if att_fused:
            need.append(lb.rs_din_att_prelu_bwd_workspace_size(B, T, 4 * K, *att.kernels[1].shape))
        gws = _gemm_ws(self, max(need))
        gw = (ptr(gws), gws.numel())

        # ---- forward, keeping what the backward needs
        hist_ids = [h.reshape(M, 1) for h in hists]
        cand_ids = [cand[:, i:i + 1] for i in range(nb)]
        item = self._behaviour_embed(cand_ids, B, check_ids)
        seq = self._behaviour_embed(hist_ids, M, check_ids)
        x = emp(B, width)
        h0 = emp(M, 4 * K)
        call("rs_din_att_concat", ptr(item), ptr(seq), B, T, K, ptr(h0), st)
        att_in, att_pre = [h0], []

        def dice_fwd(d, x, m, n):
            # Dice under fit: batch statistics (kept for the backward), moving averages moved
            mu, vr, y = emp(n), emp(n), emp(m, n)
            call("rs_dice_train_fwd", ptr(x), m, n, ptr(d.alphas), d.epsilon, 0.99, ptr(d.moving_mean),
                 ptr(d.moving_variance), ptr(mu), ptr(vr), ptr(y), *gw, st)
            return (mu, vr), y

        score = emp(M)
        if att_fused:  # the unit's forward in one launch, z1 / z2 kept
            (W1, W2), (b1, b2), (al1, al2) = att.kernels, att.biases, att.alphas
            att_pre = [emp(M, W1.shape[1]), emp(M, W2.shape[1])]
            call("rs_din_att_prelu_fwd", ptr(h0), ptr(W1), ptr(b1), ptr(al1), ptr(W2), ptr(b2), ptr(al2),
                 ptr(att.out_kernel), ptr(att.out_bias), B, T, 4 * K, W1.shape[1], W2.shape[1], ptr(att_pre[0]),
                 ptr(att_pre[1]), ptr(score), st)
        else:
            for W, b, al in zip(att.kernels, att.biases, att.alphas):
                n = W.shape[1]
                z, y = emp(M, n), emp(M, n)
                call("rs_dense_fwd", ptr(att_in[-1]), att_in[-1].stride(0), ptr(W), ptr(b), None, _lib.ACT[None],
                     ptr(z), n, M, W.shape[0], n, st)
                call("rs_prelu_rows_fwd", ptr(z), M, n, ptr(al), T, ptr(y), st)
                att_pre.append(z)
                att_in.append(y)
            for d in att.dice:  # att_attention 'dice': Dice layers on the 4k-wide concat, no Dense
                saved, y = dice_fwd(d, att_in[-1], M, 4 * K)
                att_pre.append(saved)
                att_in.append(y)
            hl = att_in[-1]
            call("rs_dense_fwd", ptr(hl), hl.stride(0), ptr(att.out_kernel), ptr(att.out_bias), None,
                 _lib.ACT[None], ptr(score), 1, M, hl.shape[1], 1, st)
        a = emp(B, T)
        h_first = hists[0]
        call("rs_masked_softmax_pool", ptr(score), ptr(h_first), _lib.id_kind(h_first), h_first.stride(0), ptr(seq),
             B, T, K, ptr(a), ptr(x), width, st)
        x[:, K:2 * K].copy_(item)
        col = 2 * K
        other_ids = []
        for f, layer in zip(self.other_sparse, self.embed_sparse_layers):
            ids = _ids_tensor(inputs[f["feat"]], dev).reshape(B, 1)
            other_ids.append(ids)
            layer.gather(ids, out=x[:, col:col + layer.k], check_ids=check_ids)
            col += layer.k
        for f in self.dense_feature_columns:
            x[:, col:col + 1] = _to_device_f32(inputs[f["feat"]], dev).reshape(B, 1)
            col += 1
        mean, var, y0 = emp(width), emp(width), emp(B, width)
        call("rs_bn_train_fwd", ptr(x), width, B, width, ptr(bn.gamma), ptr(bn.beta), bn.epsilon, 0.99,
             ptr(bn.moving_mean), ptr(bn.moving_variance), ptr(mean), ptr(var), ptr(y0), width, st)
        acts, pre, dsaved = [y0], [], []
        for L in self.dense_layer:
            z, y = emp(B, L.units), emp(B, L.units)
            call("rs_dense_fwd", ptr(acts[-1]), acts[-1].stride(0), ptr(L.kernel), ptr(L.bias), None,
                 _lib.ACT[None], ptr(z), L.units, B, L.kernel.shape[0], L.units, st)
            if L.activation == "dice":
                saved, y = dice_fwd(L.dice, z, B, L.units)
                dsaved.append(saved)
            else:
                call("rs_prelu_rows_fwd", ptr(z), B, L.units, ptr(L.alpha), 1, ptr(y), st)
                dsaved.append(None)
            pre.append(z)
            acts.append(y)
        if rate > 0:  # in place: the backward reads the layers' pre-activations, and BN's input, only
            rng = _dropout_rng(self)
            drop_off = rng.draw(acts[-1], rate, st)
        out = self.out_layer
        logit = emp(B)
        call("rs_dense_fwd", ptr(acts[-1]), acts[-1].stride(0), ptr(out.kernel), ptr(out.bias), None,
             _lib.ACT[None], ptr(logit), 1, B, out.kernel.shape[0], 1, st)
        g, g0 = emp(B), emp(B)
        loss = emp(B) if return_loss else None
        call("rs_head_grad", ptr(logit), ptr(logit), ptr(labels), B, 1.0, 0.0, ptr(g), ptr(g0), ptr(loss), st)

        # ---- backward (every gradient before any update)
        updates = []

        def dense_back(W, bias, a_in, dz, m):
            kin, n = W.shape
            dW, db, din = emp(kin, n), emp(n), emp(m, kin)
            call("rs_gemm", 1, 0, kin, n, m, 1.0, ptr(a_in), a_in.stride(0), ptr(dz), dz.stride(0), 0.0, ptr(dW), n,
                 None, 0, *gw, st)
            call("rs_col_sum_split", ptr(dz), dz.stride(0), m, n, ptr(db), *gw, st)
            call("rs_gemm", 0, 1, m, kin, n, 1.0, ptr(dz), dz.stride(0), ptr(W), n, 0.0, ptr(din), kin, None, 0,
                 *gw, st)
            updates.extend([(W, dW), (bias, db)])
            return din

        def prelu_back(z, dy, alpha, period, m):
            n = z.shape[1]
            dz, dal = emp(m, n), emp(alpha.numel())
            call("rs_prelu_rows_bwd", ptr(z), ptr(dy), m, n, ptr(alpha), period, ptr(dz), ptr(dal), *gw, st)
            updates.append((alpha, dal))
            return dz

        def dice_back(d, x, saved, dy, m, n):
            dx, dal = emp(m, n), emp(n)
            call("rs_dice_train_bwd", ptr(x), m, n, ptr(d.alphas), ptr(saved[0]), ptr(saved[1]), d.epsilon, ptr(dy),
                 ptr(dx), ptr(dal), *gw, st)
            updates.append((d.alphas, dal))
            return dx

        dh = dense_back(out.kernel, out.bias, acts[-1], g.view(B, 1), B)
        if rate > 0:
            rng.redraw(dh, rate, drop_off, st)
            rng.end_step(st)
        for li in reversed(range(len(self.dense_layer))):
            L = self.dense_layer[li]
            if L.activation == "dice":
                dz = dice_back(L.dice, pre[li], dsaved[li], dh, B, L.units)
            else:
                dz = prelu_back(pre[li], dh, L.alpha, 1, B)
            dh = dense_back(L.kernel, L.bias, acts[li], dz, B)
        dx, dgam, dbet = emp(B, width), emp(width), emp(width)
        call("rs_bn_train_bwd", ptr(x), width, B, width, ptr(mean), ptr(var), ptr(bn.gamma), bn.epsilon, ptr(dh),
             dh.stride(0), ptr(dx), width, ptr(dgam), ptr(dbet), st)
        updates.extend([(bn.gamma, dgam), (bn.beta, dbet)])
        ds, dseq = emp(M), emp(M, K)
        call("rs_masked_softmax_pool_bwd", ptr(a), ptr(h_first), _lib.id_kind(h_first), h_first.stride(0), ptr(seq),
             ptr(dx), width, B, T, K, ptr(ds), ptr(dseq), st)
        if att_fused:
            # the whole attention-unit backward in one launch (+ its partial sums)
            (W1, W2), (b1, b2), (al1, al2) = att.kernels, att.biases, att.alphas
            h1, h2 = W2.shape
            dh3 = emp(M, 4 * K)
            gr = [emp(4 * K, h1), emp(h1), emp(T, h1), emp(h1, h2), emp(h2), emp(T, h2), emp(h2), emp(1)]
            call("rs_din_att_prelu_bwd", ptr(h0), ptr(att_pre[0]), ptr(att_pre[1]), ptr(ds), ptr(W1), ptr(W2),
                 ptr(al1), ptr(al2), ptr(att.out_kernel), B, T, 4 * K, h1, h2, ptr(dh3), *[ptr(v) for v in gr], *gw,
                 st)
            updates.extend(zip([W1, b1, al1, W2, b2, al2, att.out_kernel, att.out_bias], gr))
        else:
            dh3 = dense_back(att.out_kernel, att.out_bias, hl, ds.view(M, 1), M)
            for li in reversed(range(len(att.kernels))):
                dz = prelu_back(att_pre[li], dh3, att.alphas[li], T, M)
                dh3 = dense_back(att.kernels[li], att.biases[li], att_in[li], dz, M)
        for li in reversed(range(len(att.dice))):
            dh3 = dice_back(att.dice[li], att_in[li], att_pre[li], dh3, M, 4 * K)
        call("rs_din_att_concat_bwd", ptr(dh3), ptr(item), ptr(seq), B, T, K, ptr(dx) + 4 * K, width, ptr(dseq), st)

        # ---- SGD
        _lib.sgd_update_multi([(w, gr, gr.numel(), 0.0) for w, gr in updates], lr, st)
        ws_n = _lib.lib().rs_embedding_sgd_workspace_size(M)
        ws = self.__dict__.get("_emb_ws")
        if ws is None or ws.numel() < ws_n:
            ws = self.__dict__["_emb_ws"] = torch.empty(ws_n, dtype=torch.uint8, device=dev)

        def emb_sgd(layer, ids, grad_ptr, ldg, rows):
            call("rs_embedding_sgd", ptr(layer.table), layer.total_rows, layer.k, ptr(ids), _lib.id_kind(ids),
                 ids.stride(0), ptr(layer.field_offsets), ptr(layer.field_vocab), 1, rows, grad_ptr, ldg, float(lr),
                 ptr(ws), None, st)

        col = 0
        for i, layer in enumerate(self.embed_seq_layers):
            emb_sgd(layer, hist_ids[i], ptr(dseq) + 4 * col, K, M)
            emb_sgd(layer, cand_ids[i], ptr(dx) + 4 * (K + col), width, B)
            col += layer.k
        col = 2 * K
        for layer, ids in zip(self.embed_sparse_layers, other_ids):
            emb_sgd(layer, ids, ptr(dx) + 4 * col, width, B)
            col += layer.k
        self._weights_changed()
        for L in list(self.embed_seq_layers) + list(self.embed_sparse_layers):
            L._weights_changed()
        return loss


# ------------------------------------ other CTR models
class NFM(TowerMixin, KerasModule):
    """NFM(feature_columns, hidden_units, output_dim, activation='relu',
    dropout=0) — model/nfm.py:13-33, with 3-D embeddings (documented
    deviation: on the reference's rank-2 EmbedLayer output the bi-interaction
    reduce_sum collapses to [B] and the concat with the dense block fails):
    x = BN(concat([dense, 0.5((sum_f e)^2 - sum_f e^2)])) -> DNNLayer ->
    Dense(1) -> sigmoid.  ids -> rows -> bi-interaction -> [dense | pooled]
    in one launch (rs_embed_pair_pool_fwd), BN (rs_affine_act), then the
    DNNLayer + output Dense as ONE tower launch (rs_mlp_fwd)."""

    def __init__(self, feature_columns, hidden_units, output_dim, activation="relu", dropout=0, embed_dim=8,
                 device=None, seed=None):
        super().__init__(device, seed)
        self.dense_feature_columns, self.sparse_feature_columns = feature_columns
        self.nd = len(self.dense_feature_columns)
        self.dnn_layers = DNNLayer(hidden_units, output_dim, activation, dropout, device=device,
                                   seed=_subseed(self._gen))
        self.emb_layers = EmbedLayer(self.sparse_feature_columns, embed_dim, device=device, seed=_subseed(self._gen))
        self.bn_layer = BatchNormalization(device=device)
        self.output_layer = Dense(1, activation="sigmoid", device=device, seed=_subseed(self._gen))
        d = self.nd + embed_dim
        self.dnn_layers.build(d)
        self.output_layer.build(int(output_dim))
        self.bn_layer.build(d)
        self._err = _ErrFlag(self._dev)

    def _layers(self):
        return list(self.dnn_layers.hidden_layer) + [self.dnn_layers.output_layer, self.output_layer]

    def bi_interaction_input(self, inputs, check_ids=True):
        """concat([dense, BiInteraction(emb)]) [B, nd+k] (model/nfm.py:26-29)."""
        dense, ids = _split_criteo(inputs, self.nd, self._dev)
        e = self.emb_layers
        B = ids.shape[0]
        x = torch.empty(B, self.nd + e.k, dtype=torch.float32, device=self._dev)
        call("rs_embed_pair_pool_fwd", ptr(ids), _lib.id_kind(ids), ids.stride(0), ptr(e.table),
             ptr(e.field_offsets), ptr(e.field_vocab), e.n_fields, e.k, 0, ptr(dense), dense.stride(0), self.nd,
             ptr(x), x.stride(0), self.nd, None, None, 0, None, B, ptr(self._err.t), _lib.stream())
        if check_ids:
            self._err.check("NFM")
        return x

    def forward(self, inputs, check_ids=True):
        x = self.bi_interaction_input(inputs, check_ids)
        if self.tower_ok():
            # BatchNormalization + DNNLayer + Dense(1, sigmoid) in one launch
            if self.bn_layer.gamma is None:
                self.bn_layer.build(x.shape[-1])
            return self.tower(x, in_affine=self.bn_layer.affine())
        return self.output_layer(self.dnn_layers(self.bn_layer(x)))

    def train_step(self, inputs, labels, lr=0.01, return_loss=False, check_ids=True, dropout=None):
        """One step of compile_fit on NFM (utils/compile_fit.py:9-15; the
        reference's NFM demo trains this way, model/nfm.py:47) with
        NFM.call in training mode:
          [dense | Bi-Interaction] (rs_embed_pair_pool_fwd) and the rows
          (rs_embed_gather), rs_bn_train_fwd (batch statistics, moving
          averages), the DNNLayer + output Dense with saved activations
          (rs_dense_fwd, logit), rs_head_grad, the DNN backward (rs_gemm /
          rs_col_sum), rs_bn_train_bwd, rs_bi_interaction_bwd (de_f = dbi
          (S - e_f)), SGD of the dense parameters and row-sparse
          rs_embedding_sgd.  DNNLayer's Dropout after each hidden layer
          (layer/interaction.py:44) runs in training mode as in
          DeepFM.train_step (counter-based rs_dropout masks, regenerated in
          the backward; dropout=False turns it off, a float overrides the rate).
        Returns per-sample losses (before the step) if ``return_loss``."""
        dnn = self.dnn_layers
        rate = _dropout_rate(dnn, dropout)
        _check_train_tower("NFM", dnn)
        dense, ids = _split_criteo(inputs, self.nd, self._dev)
        labels = _to_device_f32(labels, self._dev).reshape(-1)
        e, bn, out = self.emb_layers, self.bn_layer, self.output_layer
        B, F, k, st, dev = ids.shape[0], e.n_fields, e.k, _lib.stream(), self._dev
        emp = lambda *shape: torch.empty(*shape, dtype=torch.float32, device=dev)
        x = self.bi_interaction_input(inputs, check_ids)  # [B, nd + k]
        rows = e.gather(ids, check_ids=False)             # [B, F*k] (ids checked above)
        D = self.nd + k
        mean, var, y0 = emp(D), emp(D), emp(B, D)
        call("rs_bn_train_fwd", ptr(x), D, B, D, ptr(bn.gamma), ptr(bn.beta), bn.epsilon, 0.99, ptr(bn.moving_mean),
             ptr(bn.moving_variance), ptr(mean), ptr(var), ptr(y0), D, st)
        layers = self._layers()
        acts, drop = _dnn_train_forward(self, dnn, y0, rate, st)
        acts.append(dnn.output_layer(acts[-1]))
        logit = emp(B)
        call("rs_dense_fwd", ptr(acts[-1]), acts[-1].stride(0), ptr(out.kernel), ptr(out.bias), None,
             _lib.ACT[None], ptr(logit), 1, B, out.kernel.shape[0], 1, st)
        g, g0 = emp(B), emp(B)
        loss = emp(B) if return_loss else None
        call("rs_head_grad", ptr(logit), ptr(logit), ptr(labels), B, 1.0, 0.0, ptr(g), ptr(g0), ptr(loss), st)
        gws = _gemm_ws(self, max(_lib.lib().rs_gemm_workspace_size(L.kernel.shape[0], L.kernel.shape[1], B)
                                 for L in layers))
        grads, delta = _dnn_backward(layers, acts, g.view(B, 1), (ptr(gws), gws.numel()), emp, st, drop=drop)
        dx, dgam, dbet = emp(B, D), emp(D), emp(D)
        call("rs_bn_train_bwd", ptr(x), D, B, D, ptr(mean), ptr(var), ptr(bn.gamma), bn.epsilon, ptr(delta),
             delta.stride(0), ptr(dx), D, ptr(dgam), ptr(dbet), st)
        de = emp(B, F * k)
        call("rs_bi_interaction_bwd", ptr(rows), F * k, ptr(dx) + 4 * self.nd, D, F, k, B, ptr(de), F * k, st)
        _lib.sgd_update_multi(_dnn_updates(grads) + [(bn.gamma, dgam, D, 0.0), (bn.beta, dbet, D, 0.0)], lr, st)
        ws_n = _lib.lib().rs_embedding_sgd_workspace_size(B * F)
        ws = self.__dict__.get("_emb_ws")
        if ws is None or ws.numel() < ws_n:
            ws = self.__dict__["_emb_ws"] = torch.empty(ws_n, dtype=torch.uint8, device=dev)
        call("rs_embedding_sgd", ptr(e.table), e.total_rows, k, ptr(ids), _lib.id_kind(ids), ids.stride(0),
             ptr(e.field_offsets), ptr(e.field_vocab), F, B, ptr(de), F * k, float(lr), ptr(ws), None, st)
        self._weights_changed()
        return loss


class AFM(KerasModule):
    """AFM(feature_columns, mode) — model/afm.py:11-19: sigmoid(AFMLayer(x)),
    i.e. sigmoid(sigmoid(Dense(1)(pool over pairs))) — both sigmoids in the
    one rs_embed_pair_pool_fwd launch."""

    def __init__(self, feature_columns, mode, device=None, seed=None):
        super().__init__(device, seed)
        self.afm_layer = AFMLayer(feature_columns, mode, device=device, seed=_subseed(self._gen))

    def forward(self, inputs, check_ids=True):
        return self.afm_layer.pooled(inputs, check_ids, n_sigmoid=2)[1]


class FFM(KerasModule):
    """FFM(feature_columns, k, w_reg=1e-4, v_reg=1e-4) — model/ffm.py:10-22:
    sigmoid(FFMLayer(x)), one launch (rs_ffm_fwd)."""

    def __init__(self, feature_columns, k, w_reg=1e-4, v_reg=1e-4, device=None, seed=None):
        super().__init__(device, seed)
        self.dense_feature_columns, self.sparse_feature_columns = feature_columns
        self.ffm = FFMLayer(feature_columns, k, w_reg, v_reg, device=device, seed=_subseed(self._gen))

    def forward(self, inputs):
        return self.ffm.logits(inputs, n_sigmoid=1)

    def train_step(self, inputs, labels, lr=0.01, return_loss=False):
        """One step of compile_fit on FFM (utils/compile_fit.py:9-15; the
        reference's FFM demo trains this way, model/ffm.py:36): BCE on
        sigmoid(FFMLayer) plus FFMLayer's l2(w_reg) / l2(v_reg) regularisers on
        every row of w / v (layer/interaction.py:131-139), plain SGD:
          rs_ffm_train_fwd (per sample: Fm, z, g and the shared gradient row
          G = g (T - Fm)), rs_gemm / rs_col_sum (the dense rows' and w0's
          gradients), rs_l2_decay (every row of w and v), rs_sgd_update_multi (dense
          rows, w0) and rs_embedding_sgd_strided (each looked-up row of v
          gets its sample's G, of w its g; duplicates summed in lookup order).
        Out-of-range ids train nothing (tf.one_hot's zero row).  Every
        gradient comes from the pre-step weights.  Returns per-sample losses
        (before the step) if ``return_loss``."""
        L = self.ffm
        if isinstance(inputs, (tuple, list)):
            dense, ids = _to_device_f32(inputs[0], self._dev), _ids_tensor(inputs[1], self._dev)
        else:
            X = _to_device_f32(inputs, self._dev)
            dense, ids = X[:, :L.nd], X[:, L.nd:]
        labels = _to_device_f32(labels, self._dev).reshape(-1)
        B, F, k, nd, st, dev = ids.shape[0], len(L.onehot_dims), L.k, L.nd, _lib.stream(), self._dev
        E = L.field_num * k
        emp = lambda *shape: torch.empty(*shape, dtype=torch.float32, device=dev)
        G, g = emp(B, E), emp(B)
        loss = emp(B) if return_loss else None
        call("rs_ffm_train_fwd", ptr(ids), _lib.id_kind(ids), ids.stride(0), ptr(dense), dense.stride(0), nd,
             ptr(L.v), ptr(L.w), ptr(L.w0), ptr(L.field_offsets), ptr(L.field_vocab), F, k, ptr(labels), B, ptr(G),
             ptr(g), ptr(loss), st)
        gws = _gemm_ws(self, max(_lib.lib().rs_gemm_workspace_size(nd, E, B), _lib.lib().rs_gemm_workspace_size(nd, 1, B)))
        gw = (ptr(gws), gws.numel())
        dvd, dwd, dw0 = emp(max(nd, 1), E), emp(max(nd, 1)), emp(1)
        if nd:
            call("rs_gemm", 1, 0, nd, E, B, 1.0, ptr(dense), dense.stride(0), ptr(G), E, 0.0, ptr(dvd), E, None, 0,
                 *gw, st)
            call("rs_gemm", 1, 0, nd, 1, B, 1.0, ptr(dense), dense.stride(0), ptr(g), 1, 0.0, ptr(dwd), 1, None, 0,
                 *gw, st)
        call("rs_col_sum", ptr(g), 1, B, 1, ptr(dw0), st)
        # l2 on every row (old weights), then the data gradients
        call("rs_l2_decay", ptr(L.v), L.v.numel(), float(lr), float(L.v_reg), st)
        call("rs_l2_decay", ptr(L.w), L.w.numel(), float(lr), float(L.w_reg), st)
        _lib.sgd_update_multi(([(L.v, dvd, nd * E, 0.0), (L.w, dwd, nd, 0.0)] if nd else []) + [(L.w0, dw0, 1, 0.0)],
                              lr, st)
        n_sparse = L.feature_num - nd
        ws_n = _lib.lib().rs_embedding_sgd_workspace_size(B * F)
        ws = self.__dict__.get("_emb_ws")
        if ws is None or ws.numel() < ws_n:
            ws = self.__dict__["_emb_ws"] = torch.empty(ws_n, dtype=torch.uint8, device=dev)
        call("rs_embedding_sgd_strided", ptr(L.v) + 4 * nd * E, n_sparse, E, ptr(ids), _lib.id_kind(ids),
             ids.stride(0), ptr(L.field_offsets), ptr(L.field_vocab), F, B, ptr(G), E, 0, float(lr), ptr(ws), None,
             st)
        call("rs_embedding_sgd_strided", ptr(L.w) + 4 * nd, n_sparse, 1, ptr(ids), _lib.id_kind(ids), ids.stride(0),
             ptr(L.field_offsets), ptr(L.field_vocab), F, B, ptr(g), 1, 0, float(lr), ptr(ws), None, st)
        self._weights_changed()
        return loss
