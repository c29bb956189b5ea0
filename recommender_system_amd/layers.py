"""Keras-Layer-compatible modules for the CTR forward path, on librs_hip.so.

Each class keeps the reference layer's name, constructor arguments and
``call`` semantics (Hcyand/recommender_system, algorithm/deep_learning/layer/):

  EmbedLayer(sparse_feature_columns, k=8)     layer/core.py:267-280
  FMLayer(k, reg_w=1e-4, reg_b=1e-4)          layer/interaction.py:86-114
  CrossLayer(layer_num, reg_w, reg_b)         layer/interaction.py:49-83
  InnerProductLayer()                         layer/interaction.py:166-183
  DNNLayer(hidden_units, output_dim, activation='relu', dropout=0.2)
                                              layer/interaction.py:30-46
  Attention(hidden_units, activation='prelu') layer/interaction.py:355-406
  Dice(axis=-1, epsilon=1e-9)                 layer/interaction.py:410-425
  Dense / PReLU / BatchNormalization          the Keras layers the models use

Weights are built lazily on the first call from the input shape, like Keras
``build``, with the reference's initializers (Embedding U(-0.05,0.05),
random_normal N(0,0.05), glorot_uniform kernels, zero biases, zero PReLU/Dice
alphas, BN moving stats 0/1), and are stored in Keras orientation (Dense
kernel (in, out)).  ``keras_weights()`` / ``set_keras_weights()`` exchange them
by Keras weight name.

The forward path is inference only (Dropout is the identity, BN uses moving
statistics) and runs only on HIP device tensors through the C-ABI kernels:
there is no CPU fallback — a CPU tensor is an error.  An embedding id outside
[0, vocab) raises IndexError as TF's CPU Embedding does (the check costs one
device sync; pass ``check_ids=False`` to skip the host-side raise).
"""
from __future__ import annotations

import ctypes as C
import math
from typing import Sequence

import torch
from torch import nn

from . import _lib
from ._lib import call, ptr

_DEFAULT_DEVICE = "cuda"


def _device(device):
    return torch.device(device if device is not None else _DEFAULT_DEVICE)


def _stream():
    return _lib.stream()


def _to_device_f32(x, device):
    t = torch.as_tensor(x)
    if t.dtype != torch.float32:
        t = t.to(torch.float32)  # Keras Model.__call__ autocast of float inputs
    return t.to(device).contiguous()


def _ids_tensor(ids, device):
    t = torch.as_tensor(ids)
    if t.dtype == torch.float64:
        t = t.to(torch.float32)  # autocast first, then the Embedding's int cast in-kernel
    if t.dtype not in (torch.int32, torch.int64, torch.float32):
        t = t.to(torch.int64)
    return t.to(device)


class _ErrFlag:
    """Device int flag the kernels OR rs_flag bits into: an out-of-range id
    (IndexError, as TF's Embedding raises) or a kernel-internal failure."""

    def __init__(self, device):
        self.t = torch.zeros(1, dtype=torch.int32, device=device)

    def check(self, what):
        v = int(self.t.item())
        if v != 0:
            self.t.zero_()
            if v & ~_lib.FLAG_BAD_ID:
                raise _lib.RSError(f"{what}: kernel error flag {v:#x} ({_lib.flag_names(v)})")
            raise IndexError(f"{what}: embedding id out of range (indices must be in [0, vocab))")


def _glorot_uniform(fan_in, fan_out, gen, device):
    lim = math.sqrt(6.0 / (fan_in + fan_out))
    return (torch.rand(fan_in, fan_out, generator=gen, device="cpu") * 2 - 1).mul_(lim).to(device)


def _normal(shape, gen, device, std=0.05):
    return torch.randn(*shape, generator=gen, device="cpu").mul_(std).to(device)


class KerasModule(nn.Module):
    """Base: Keras-named weight exchange and a seeded CPU generator for init."""

    def __init__(self, device=None, seed=None):
        super().__init__()
        self._dev = _device(device)
        self._gen = torch.Generator(device="cpu")
        self._gen.manual_seed(seed if seed is not None else torch.initial_seed() % (2 ** 31))

    def keras_weights(self) -> dict:
        return {n: p for n, p in self.named_parameters()}

    def set_keras_weights(self, weights: dict, strict: bool = True):
        own = dict(self.named_parameters())
        for name, val in weights.items():
            if name not in own:
                if strict:
                    raise KeyError(f"unknown weight {name!r}; have {sorted(own)}")
                continue
            v = torch.as_tensor(val, dtype=torch.float32).reshape(own[name].shape)
            with torch.no_grad():
                own[name].copy_(v.to(own[name].device))
        if strict:
            missing = set(own) - set(weights)
            if missing:
                raise KeyError(f"missing weights {sorted(missing)}")
        self._weights_changed()

    def _weights_changed(self):
        for m in self.modules():
            if m is not self and isinstance(m, KerasModule):
                m._invalidate()
        self._invalidate()

    def _invalidate(self):
        pass


# --------------------------------------------------------------- embedding
class EmbedLayer(KerasModule):
    """EmbedLayer(sparse_feature_columns, k=8) — layer/core.py:267-280.

    One Keras ``Embedding(feat_onehot_dim, k)`` per sparse field, stored as ONE
    contiguous [sum(vocab), k] HBM table (64-B rows at k=16) with per-field row
    offsets; ``field_table(i)`` is field i's Embedding matrix (a view).
    ``forward(sparse)`` returns the flattened [B, F*k] (field-major), exactly
    like the reference (which ignores feat['embed_dim'] and uses k).
    """

    def host_meta(self):
        """(offsets, vocab) as host int64 arrays (addresses), for the entry
        points that take the field metadata by value."""
        return C.addressof(self._host_offsets), C.addressof(self._host_vocab)

    def __init__(self, sparse_feature_columns, k=8, device=None, seed=None):
        super().__init__(device, seed)
        self.k = int(k)
        self.vocab_sizes = [int(f["feat_onehot_dim"]) for f in sparse_feature_columns]
        self.n_fields = len(self.vocab_sizes)
        offs = [0]
        for v in self.vocab_sizes[:-1]:
            offs.append(offs[-1] + v)
        self.row_offsets = offs
        self.total_rows = sum(self.vocab_sizes)
        self.register_buffer("field_offsets", torch.tensor(offs, dtype=torch.int64, device=self._dev))
        self.register_buffer("field_vocab", torch.tensor(self.vocab_sizes, dtype=torch.int64, device=self._dev))
        # host copies of the same metadata (rs_embed_fm_fwd_hm: kernel arguments)
        F = max(self.n_fields, 1)
        self._host_offsets = (C.c_int64 * F)(*offs[:self.n_fields])
        self._host_vocab = (C.c_int64 * F)(*self.vocab_sizes)
        table = torch.empty(self.total_rows, self.k, dtype=torch.float32, device=self._dev)
        if table.is_cuda:
            g = torch.Generator(device=table.device)
            g.manual_seed(int(torch.randint(0, 2 ** 31, (1,), generator=self._gen)))
            table.uniform_(-0.05, 0.05, generator=g)
        else:
            table.uniform_(-0.05, 0.05, generator=self._gen)
        self.table = nn.Parameter(table, requires_grad=False)
        self._err = _ErrFlag(self._dev)

    def field_table(self, i: int) -> torch.Tensor:
        o = self.row_offsets[i]
        return self.table[o:o + self.vocab_sizes[i]]

    def keras_weights(self):
        return {f"embedding_{i}/embeddings": self.field_table(i) for i in range(self.n_fields)}

    def set_keras_weights(self, weights, strict=True):
        for i in range(self.n_fields):
            name = f"embedding_{i}/embeddings"
            if name in weights:
                with torch.no_grad():
                    self.field_table(i).copy_(torch.as_tensor(weights[name], dtype=torch.float32).to(self._dev))
            elif strict:
                raise KeyError(f"missing weight {name}")

    def gather(self, ids, dense=None, out=None, check_ids=True):
        """x = [dense | emb] in one launch (rs_embed_gather)."""
        ids = _ids_tensor(ids, self._dev)
        B = ids.shape[0]
        nd = 0 if dense is None else dense.shape[1]
        d = nd + self.n_fields * self.k
        if out is None:
            out = torch.empty(B, d, dtype=torch.float32, device=self._dev)
        call("rs_embed_gather", ptr(ids), _lib.id_kind(ids), ids.stride(0), ptr(dense),
             0 if dense is None else dense.stride(0), nd, ptr(self.table), ptr(self.field_offsets),
             ptr(self.field_vocab), self.n_fields, self.k, ptr(out), out.stride(0), B, ptr(self._err.t), _stream())
        if check_ids:
            self._err.check("EmbedLayer")
        return out

    def forward(self, inputs, check_ids=True):
        if inputs.shape[1] != self.n_fields:
            raise ValueError(f"EmbedLayer expects {self.n_fields} sparse columns, got {inputs.shape[1]}")
        return self.gather(inputs, check_ids=check_ids)


# ---------------------------------------------------------------------- FM
class FMLayer(KerasModule):
    """FMLayer(k, reg_w=1e-4, reg_b=1e-4) — layer/interaction.py:86-114.

    Weights w0:(1,) zeros, w1:(n,1) and v:(n,k) ~ N(0, 0.05), built from the
    input width on the first call.  The regularisers only affect training
    losses and are kept as attributes.  ``forward(x[B,n]) -> [B,1]``.
    """

    def __init__(self, k, reg_w=1e-4, reg_b=1e-4, device=None, seed=None, input_dim=None):
        super().__init__(device, seed)
        self.k = int(k)
        self.reg_w, self.reg_b = reg_w, reg_b
        self.w0 = self.w1 = self.v = None
        self._prep = None
        self._prep_key = None
        if input_dim is not None:
            self.build(input_dim)

    def build(self, n):
        self.w0 = nn.Parameter(torch.zeros(1, device=self._dev), requires_grad=False)
        self.w1 = nn.Parameter(_normal((n, 1), self._gen, self._dev), requires_grad=False)
        self.v = nn.Parameter(_normal((n, self.k), self._gen, self._dev), requires_grad=False)
        self._invalidate()

    @property
    def built(self):
        return self.v is not None

    def _invalidate(self):
        self._prep = None
        self._prep_key = None

    def prepared(self, nd, n_fields, emb_k):
        """Packed MFMA operand image of (w1, v) for a given x layout."""
        key = (nd, n_fields, emb_k, self.w1._version, self.v._version, self.w1.data_ptr(), self.v.data_ptr())
        if self._prep is None or self._prep_key != key:
            n = _lib.lib().rs_fm_prepared_size(nd, n_fields, emb_k, self.k)
            if n <= 0:
                raise ValueError("FMLayer: unsupported shape")
            self._prep = torch.empty(n, dtype=torch.float32, device=self._dev)
            call("rs_fm_prepare", ptr(self.w1), ptr(self.v), nd, n_fields, emb_k, self.k, ptr(self._prep), _stream())
            self._prep_key = key
        return self._prep

    def forward(self, inputs):
        x = _to_device_f32(inputs, self._dev)
        if not self.built:
            self.build(x.shape[-1])
        B, n = x.shape
        if n != self.w1.shape[0]:
            raise ValueError(f"FMLayer built for {self.w1.shape[0]} inputs, got {n}")
        out = torch.empty(B, 1, dtype=torch.float32, device=self._dev)
        prep = self.prepared(n, 0, 0)
        call("rs_fm_fwd", ptr(x), x.stride(0), n, ptr(prep), ptr(self.w0), self.k, ptr(out), B, _stream())
        return out


# --------------------------------------------------------------- DCN cross
class CrossLayer(KerasModule):
    """CrossLayer(layer_num, reg_w=1e-4, reg_b=1e-4) — layer/interaction.py:49-83.
    Weights w{i}, b{i}: (d,1) ~ N(0, 0.05).  ``forward(x[B,d]) -> [B,d]``."""

    def __init__(self, layer_num, reg_w=1e-4, reg_b=1e-4, device=None, seed=None, input_dim=None):
        super().__init__(device, seed)
        self.layer_num = int(layer_num)
        self.reg_w, self.reg_b = reg_w, reg_b
        self.cross_weight = nn.ParameterList()
        self.cross_bias = nn.ParameterList()
        self._prep = None
        self._prep_key = None
        if input_dim is not None:
            self.build(input_dim)

    def build(self, d):
        for _ in range(self.layer_num):
            self.cross_weight.append(nn.Parameter(_normal((d, 1), self._gen, self._dev), requires_grad=False))
        for _ in range(self.layer_num):
            self.cross_bias.append(nn.Parameter(_normal((d, 1), self._gen, self._dev), requires_grad=False))
        self._invalidate()

    @property
    def built(self):
        return len(self.cross_weight) == self.layer_num and (self.layer_num == 0 or len(self.cross_bias) > 0)

    def keras_weights(self):
        out = {f"w{i}": w for i, w in enumerate(self.cross_weight)}
        out.update({f"b{i}": b for i, b in enumerate(self.cross_bias)})
        return out

    def set_keras_weights(self, weights, strict=True):
        for i in range(self.layer_num):
            with torch.no_grad():
                self.cross_weight[i].copy_(torch.as_tensor(weights[f"w{i}"], dtype=torch.float32).reshape(-1, 1))
                self.cross_bias[i].copy_(torch.as_tensor(weights[f"b{i}"], dtype=torch.float32).reshape(-1, 1))
        self._invalidate()

    def _invalidate(self):
        self._prep = None
        self._prep_key = None

    def prepared(self, d):
        key = tuple((p._version, p.data_ptr()) for p in list(self.cross_weight) + list(self.cross_bias))
        if self._prep is None or self._prep_key != key:
            L = self.layer_num
            n = _lib.lib().rs_cross_prepared_size(d, L)
            self._prep = torch.empty(n, dtype=torch.float32, device=self._dev)
            if L:
                W = torch.stack([w.reshape(-1) for w in self.cross_weight]).contiguous()
                Bb = torch.stack([b.reshape(-1) for b in self.cross_bias]).contiguous()
            else:
                W = Bb = None
            call("rs_cross_prepare", ptr(W), ptr(Bb), d, L, ptr(self._prep), _stream())
            self._keep = (W, Bb)  # stream-ordered lifetime
            self._prep_key = key
        return self._prep

    def forward(self, inputs, out=None):
        x = _to_device_f32(inputs, self._dev)
        if not self.built:
            self.build(x.shape[1])
        B, d = x.shape
        if out is None:
            out = torch.empty(B, d, dtype=torch.float32, device=self._dev)
        call("rs_cross_fwd", ptr(x), x.stride(0), d, self.layer_num, ptr(self.prepared(d)), ptr(out), out.stride(0),
             B, _stream())
        return out


# ------------------------------------------------------ PNN inner product
class InnerProductLayer(KerasModule):
    """InnerProductLayer() — layer/interaction.py:166-183.
    ``forward(e[B,F,k]) -> [B, F(F-1)/2]``, pairs (i<j) row-major."""

    def __init__(self, device=None):
        super().__init__(device)

    def forward(self, inputs, out=None):
        e = _to_device_f32(inputs, self._dev)
        B, F, k = e.shape
        P = F * (F - 1) // 2
        if out is None:
            out = torch.empty(B, P, dtype=torch.float32, device=self._dev)
        call("rs_inner_product_fwd", ptr(e), F, k, ptr(out), out.stride(0), B, _stream())
        return out


class OuterProductLayer(KerasModule):
    """OuterProductLayer() — layer/interaction.py:186-215.  Weight W:
    (k, P, k) ~ N(0, 0.05) (tf.random_normal_initializer()), built on the
    first call.  ``forward(e[B,F,k]) -> [B,P]`` with
    out[b,p] = sum_{a,j} e[b,row_p,j] W[a,p,j] e[b,col_p,a]."""

    def __init__(self, device=None, seed=None):
        super().__init__(device, seed)
        self.W = None
        self.field_num = self.k = None

    def build(self, F, k):
        self.field_num, self.k = int(F), int(k)
        P = F * (F - 1) // 2
        self.W = nn.Parameter(_normal((k, P, k), self._gen, self._dev), requires_grad=False)

    def keras_weights(self):
        return {"W": self.W}

    def set_keras_weights(self, weights, strict=True):
        with torch.no_grad():
            self.W.copy_(torch.as_tensor(weights["W"], dtype=torch.float32).reshape(self.W.shape))

    def _invalidate(self):
        self._prep_key = None  # W moved through a raw pointer (training): repack

    def prepared(self):
        """W packed into per-lane MFMA fragments (rs_outer_prepare), cached."""
        key = (self.W._version, self.W.data_ptr())
        if getattr(self, "_prep_key", None) != key:
            n = _lib.lib().rs_outer_prepared_size(self.field_num, self.k)
            if n < 0:
                _lib.check(-1, "rs_outer_prepared_size")
            self._prep = torch.empty(n, dtype=torch.float32, device=self._dev)
            call("rs_outer_prepare", ptr(self.W), self.field_num, self.k, ptr(self._prep), _stream())
            self._prep_key = key
        return self._prep

    def forward(self, inputs, out=None):
        e = _to_device_f32(inputs, self._dev)
        B, F, k = e.shape
        if self.W is None:
            self.build(F, k)
        if (F, k) != (self.field_num, self.k):
            raise ValueError(f"OuterProductLayer built for F={self.field_num}, k={self.k}; got {F}, {k}")
        P = F * (F - 1) // 2
        if out is None:
            out = torch.empty(B, P, dtype=torch.float32, device=self._dev)
        call("rs_outer_product_fwd", ptr(e.contiguous()), F, k, ptr(self.prepared()), ptr(out), out.stride(0), B,
             _stream())
        return out


# -------------------------------------------------------------- dense / MLP
_MLP_MAXL, _MLP_MAXD = 8, 1024  # rs_mlp_fwd limits (mlp.hip)
_ACTS = ("relu", "prelu", "sigmoid", "linear", None, "dice")


class Dense(KerasModule):
    """Keras Dense(units, activation) on 2-D inputs: kernel (in, units)
    glorot-uniform, bias zeros.  activation: None/'linear', 'relu', 'sigmoid',
    'prelu' (Keras PReLU(): alpha shape [units], zeros) or 'dice' (Dice())."""

    def __init__(self, units, activation=None, device=None, seed=None, input_dim=None):
        super().__init__(device, seed)
        if activation not in _ACTS:
            raise ValueError(f"unsupported activation {activation!r}")
        self.units = int(units)
        self.activation = activation
        self.kernel = self.bias = self.alpha = None
        self.dice = None
        if input_dim is not None:
            self.build(input_dim)

    def build(self, n):
        self.kernel = nn.Parameter(_glorot_uniform(n, self.units, self._gen, self._dev), requires_grad=False)
        self.bias = nn.Parameter(torch.zeros(self.units, device=self._dev), requires_grad=False)
        if self.activation == "prelu":
            self.alpha = nn.Parameter(torch.zeros(self.units, device=self._dev), requires_grad=False)
        if self.activation == "dice":
            self.dice = Dice(device=self._dev)
            self.dice.build(self.units)

    def keras_weights(self):
        out = {"kernel": self.kernel, "bias": self.bias}
        if self.alpha is not None:
            out["alpha"] = self.alpha
        if self.dice is not None:
            out.update({f"dice/{k}": v for k, v in self.dice.keras_weights().items()})
        return out

    def set_keras_weights(self, weights, strict=True):
        with torch.no_grad():
            self.kernel.copy_(torch.as_tensor(weights["kernel"], dtype=torch.float32))
            self.bias.copy_(torch.as_tensor(weights["bias"], dtype=torch.float32))
            if self.alpha is not None:
                self.alpha.copy_(torch.as_tensor(weights["alpha"], dtype=torch.float32).reshape(-1))
        if self.dice is not None:
            self.dice.set_keras_weights({k[5:]: v for k, v in weights.items() if k.startswith("dice/")}, strict)

    def forward(self, inputs, out=None):
        x = _to_device_f32(inputs, self._dev) if not (torch.is_tensor(inputs) and inputs.is_cuda) else inputs
        if self.kernel is None:
            self.build(x.shape[-1])
        M, K = x.shape
        if out is None:
            out = torch.empty(M, self.units, dtype=torch.float32, device=self._dev)
        act = 0 if self.activation == "dice" else _lib.ACT[self.activation]
        call("rs_dense_fwd", ptr(x), x.stride(0), ptr(self.kernel), ptr(self.bias), ptr(self.alpha), act, ptr(out),
             out.stride(0), M, K, self.units, _stream())
        if self.activation == "dice":
            out = self.dice(out, out=out)
        return out


class TowerMixin:
    """A stack of Keras Dense layers run as ONE rs_mlp_fwd launch (mlp.hip):
    activations stay in LDS, weights are packed once.  The host class
    provides ``_layers()`` (the Dense layers in order) and ``_dev``."""

    def _invalidate(self):
        # packed images keyed on tensor versions miss in-place kernel updates
        # (training steps): drop them
        self.__dict__.pop("_tower_prep", None)

    def tower_ok(self):
        ls = self._layers()
        if not (ls[0].kernel is not None and len(ls) <= _MLP_MAXL and all(l.activation != "dice" for l in ls)
                and all(d <= _MLP_MAXD for d in self._dims())):
            return False
        dims = self._dims()
        return _lib.lib().rs_mlp_prepared_size(len(ls), (C.c_int * len(dims))(*dims)) >= 0  # LDS budget

    def _dims(self):
        ls = self._layers()
        return [ls[0].kernel.shape[0]] + [l.units for l in ls]

    def prepared(self, in_rows=None):
        """Weights packed in MFMA B-fragment order (rs_mlp_prepare), cached
        until any weight changes (in-place updates bump tensor versions)."""
        params = [p for l in self._layers() for p in (l.kernel, l.bias, l.alpha) if p is not None]
        key = (tuple((p._version, p.data_ptr()) for p in params),
               None if in_rows is None else in_rows._version)
        cache = self.__dict__.setdefault("_tower_prep", {})
        slot = None if in_rows is None else in_rows.data_ptr()
        ent = cache.get(slot)
        if ent is None or ent[0] != key:
            ls = self._layers()
            dims = self._dims()
            n = len(ls)
            ci = (C.c_int * (n + 1))(*dims)
            pa = lambda ts: (C.c_void_p * n)(*[ptr(t) for t in ts])
            size = _lib.lib().rs_mlp_prepared_size(n, ci)
            if size < 0:
                _lib.check(-1, "rs_mlp_prepared_size")
            prep = torch.empty(size, dtype=torch.float32, device=self._dev)
            call("rs_mlp_prepare", n, ci, pa([l.kernel for l in ls]), pa([l.bias for l in ls]),
                 pa([l.alpha for l in ls]), ptr(in_rows), ptr(prep), _stream())
            ent = cache[slot] = (key, prep, in_rows)  # in_rows kept alive with its packing
        return ent[1]

    def tower(self, x, extra=None, c0=1.0, c1=1.0, head=False, out=None, in_affine=None):
        """rs_mlp_fwd on x:[M, K] (device, row stride x.stride(0)).  head=True:
        sigmoid(c0*dnn + c1*extra) (output_dim 1).  in_affine=(scale, shift):
        the tower runs on x * scale + shift (an inference BatchNormalization
        folded into the launch: rs_mlp_affine_fwd)."""
        ls = self._layers()
        n = len(ls)
        dims = self._dims()
        M = x.shape[0]
        if out is None:
            out = torch.empty(M, 1 if head else dims[-1], dtype=torch.float32, device=self._dev)
        acts = [_lib.ACT[l.activation] for l in ls]
        if in_affine is not None:
            sc, sh = in_affine
            if sc.numel() != dims[0] or sh.numel() != dims[0]:
                raise ValueError(f"tower: in_affine needs {dims[0]} scales and shifts")
            call("rs_mlp_affine_fwd", ptr(x), x.stride(0), ptr(sc), ptr(sh), n, (C.c_int * (n + 1))(*dims),
                 (C.c_int * n)(*acts), ptr(self.prepared()), ptr(out), out.stride(0), 1 if head else 0, ptr(extra),
                 float(c0), float(c1), M, _stream())
            return out
        call("rs_mlp_fwd", ptr(x), x.stride(0), n, (C.c_int * (n + 1))(*dims), (C.c_int * n)(*acts),
             ptr(self.prepared()), ptr(out), out.stride(0), 1 if head else 0, ptr(extra), float(c0), float(c1), M,
             _stream())
        return out


class DNNLayer(TowerMixin, KerasModule):
    """DNNLayer(hidden_units, output_dim, activation='relu', dropout=0.2) —
    layer/interaction.py:30-46.  Dropout is inactive at inference."""

    def __init__(self, hidden_units, output_dim, activation="relu", dropout=0.2, device=None, seed=None):
        super().__init__(device, seed)
        self.dropout = dropout
        self.hidden_layer = nn.ModuleList(
            [Dense(u, activation=activation, device=device, seed=int(torch.randint(0, 2 ** 31, (1,), generator=self._gen)))
             for u in hidden_units])
        self.output_layer = Dense(output_dim, activation=None, device=device,
                                  seed=int(torch.randint(0, 2 ** 31, (1,), generator=self._gen)))

    def _layers(self):
        return list(self.hidden_layer) + [self.output_layer]

    def keras_weights(self):
        out = {}
        for i, l in enumerate(self.hidden_layer):
            out.update({f"dense_{i}/{k}": v for k, v in l.keras_weights().items()})
        out.update({f"dense_out/{k}": v for k, v in self.output_layer.keras_weights().items()})
        return out

    def set_keras_weights(self, weights, strict=True):
        for i, l in enumerate(self.hidden_layer):
            l.set_keras_weights({k.split("/", 1)[1]: v for k, v in weights.items() if k.startswith(f"dense_{i}/")},
                                strict)
        self.output_layer.set_keras_weights(
            {k.split("/", 1)[1]: v for k, v in weights.items() if k.startswith("dense_out/")}, strict)

    def build(self, n):
        for layer in self.hidden_layer:
            layer.build(n)
            n = layer.units
        self.output_layer.build(n)

    def forward(self, inputs):
        x = inputs
        if torch.is_tensor(x) and x.is_cuda and x.dim() == 2 and x.stride(1) == 1 and self.output_layer.kernel is not None \
                and self.tower_ok():
            return self.tower(x)
        for layer in self.hidden_layer:
            x = layer(x)
        return self.output_layer(x)


class Dice(KerasModule):
    """Dice(axis=-1, epsilon=1e-9) at inference — layer/interaction.py:410-425:
    BN(center=False, scale=False) with moving stats, p = sigmoid(xhat),
    y = alpha*(1-p)*x + p*x.  alpha, moving_mean: zeros; moving_variance: ones."""

    def __init__(self, axis=-1, epsilon=1e-9, device=None):
        super().__init__(device)
        if axis != -1:
            raise NotImplementedError("Dice: only axis=-1 (the reference default) is supported")
        self.axis, self.epsilon = axis, float(epsilon)
        self.alphas = self.moving_mean = self.moving_variance = None

    def build(self, n):
        self.alphas = nn.Parameter(torch.zeros(n, device=self._dev), requires_grad=False)
        self.moving_mean = nn.Parameter(torch.zeros(n, device=self._dev), requires_grad=False)
        self.moving_variance = nn.Parameter(torch.ones(n, device=self._dev), requires_grad=False)

    def keras_weights(self):
        return {"dice_alpha": self.alphas, "bn/moving_mean": self.moving_mean,
                "bn/moving_variance": self.moving_variance}

    def set_keras_weights(self, weights, strict=True):
        with torch.no_grad():
            for name, p in self.keras_weights().items():
                if name in weights:
                    p.copy_(torch.as_tensor(weights[name], dtype=torch.float32).reshape(-1))
                elif strict:
                    raise KeyError(name)

    def forward(self, inputs, out=None):
        x = _to_device_f32(inputs, self._dev) if not (torch.is_tensor(inputs) and inputs.is_cuda) else inputs
        if self.alphas is None:
            self.build(x.shape[-1])
        if x.dim() != 2:
            raise NotImplementedError("Dice.forward: 2-D inputs (3-D Dice runs fused in Attention)")
        M, N = x.shape
        if out is None:
            out = torch.empty_like(x)
        call("rs_dice_fwd", ptr(x), x.stride(0), ptr(self.moving_mean), ptr(self.moving_variance),
             self.epsilon, ptr(self.alphas), ptr(out), out.stride(0), M, N, _stream())
        return out


class BatchNormalization(KerasModule):
    """Keras BatchNormalization() at inference (model/din.py:47,89):
    y = x*inv + (beta - mean*inv), inv = gamma*rsqrt(var + eps), eps 1e-3."""

    def __init__(self, epsilon=1e-3, device=None):
        super().__init__(device)
        self.epsilon = float(epsilon)
        self.gamma = self.beta = self.moving_mean = self.moving_variance = None

    def build(self, n):
        d = self._dev
        self.gamma = nn.Parameter(torch.ones(n, device=d), requires_grad=False)
        self.beta = nn.Parameter(torch.zeros(n, device=d), requires_grad=False)
        self.moving_mean = nn.Parameter(torch.zeros(n, device=d), requires_grad=False)
        self.moving_variance = nn.Parameter(torch.ones(n, device=d), requires_grad=False)

    def keras_weights(self):
        return {"gamma": self.gamma, "beta": self.beta, "moving_mean": self.moving_mean,
                "moving_variance": self.moving_variance}

    def set_keras_weights(self, weights, strict=True):
        with torch.no_grad():
            for name, p in self.keras_weights().items():
                p.copy_(torch.as_tensor(weights[name], dtype=torch.float32).reshape(-1))

    def _invalidate(self):
        self._aff_key = None  # statistics / affine moved through raw pointers (training)

    def affine(self):
        """(inv, shift) = (gamma rsqrt(var + eps), beta - mean inv), cached per
        parameter version (inference calls launch no elementwise kernels)."""
        ps = (self.gamma, self.beta, self.moving_mean, self.moving_variance)
        key = tuple((q._version, q.data_ptr()) for q in ps)
        if getattr(self, "_aff_key", None) != key:
            inv = torch.rsqrt(self.moving_variance + self.epsilon) * self.gamma
            self._aff = (inv, self.beta - self.moving_mean * inv)
            self._aff_key = key
        return self._aff

    def forward(self, x, out=None):
        if self.gamma is None:
            self.build(x.shape[-1])
        inv, shift = self.affine()
        M, N = x.shape
        if out is None:
            out = torch.empty_like(x)
        call("rs_affine_act", ptr(x), x.stride(0), ptr(inv), ptr(shift), None, 0, ptr(out), out.stride(0), M, N,
             _stream())
        return out


# ------------------------------------------------------------ DIN attention
class Attention(KerasModule):
    """Attention(hidden_units, activation='prelu') — layer/interaction.py:355-406.

    'prelu': Dense(h, PReLU()) per hidden unit count; the PReLU sits on a 3-D
    input so its alpha has shape [T, h] (Keras shared_axes=None), built on the
    first call.  'dice': len(hidden_units) Dice layers on the 4k-wide concat and
    NO Dense (exactly as the reference, :363-364).  Then Dense(1).
    ``forward([query[B,k], key[B,T,k], value[B,T,k], mask[B,T]]) -> [B,k]``.
    """

    def __init__(self, hidden_units, activation="prelu", device=None, seed=None):
        super().__init__(device, seed)
        if activation not in ("prelu", "dice"):
            raise ValueError(f"Attention activation must be 'prelu' or 'dice', got {activation!r}")
        self.hidden_units = tuple(int(h) for h in hidden_units)
        self.activation = activation
        self.kernels = nn.ParameterList()
        self.biases = nn.ParameterList()
        self.alphas = nn.ParameterList()
        self.dice = nn.ModuleList()
        self.out_kernel = self.out_bias = None
        self.T = None

    def build(self, T, k):
        self.T = T
        n = 4 * k
        if self.activation == "prelu":
            for h in self.hidden_units:
                self.kernels.append(nn.Parameter(_glorot_uniform(n, h, self._gen, self._dev), requires_grad=False))
                self.biases.append(nn.Parameter(torch.zeros(h, device=self._dev), requires_grad=False))
                self.alphas.append(nn.Parameter(torch.zeros(T, h, device=self._dev), requires_grad=False))
                n = h
        else:
            for _ in self.hidden_units:
                d = Dice(device=self._dev)
                d.build(4 * k)
                self.dice.append(d)
        self.out_kernel = nn.Parameter(_glorot_uniform(n, 1, self._gen, self._dev), requires_grad=False)
        self.out_bias = nn.Parameter(torch.zeros(1, device=self._dev), requires_grad=False)

    def fused_ok(self, k):
        """The one-launch MFMA kernel (rs_din_attention_fwd) takes the shape:
        the reference's two hidden layers, H <= 128, k in {4, 8, 16, 32}.
        Other depths / sizes run the generic path (rs_din_attention_gen_fwd)."""
        return (self.activation == "prelu" and len(self.hidden_units) == 2 and k in (4, 8, 16, 32)
                and max(self.hidden_units) <= 128)

    def ids_ok(self, k):
        """The id-driven fused path (rs_din_attention_ids_fwd) supports it."""
        return (self.activation == "prelu" and self.out_kernel is not None and len(self.hidden_units) == 2
                and k in (4, 8, 16) and self.hidden_units[0] <= 128 and self.hidden_units[1] <= 64)

    def _invalidate(self):
        self._ids_key = None  # weights moved through raw pointers (training): repack

    def prepared_ids(self, k):
        params = list(self.kernels) + list(self.biases) + list(self.alphas) + [self.out_kernel, self.out_bias]
        key = (k, self.T) + tuple((p._version, p.data_ptr()) for p in params)
        if getattr(self, "_ids_key", None) != key:
            h1, h2 = self.hidden_units
            n = _lib.lib().rs_din_prepared_size(self.T, k, h1, h2)
            if n < 0:
                _lib.check(-1, "rs_din_prepared_size")
            prep = torch.empty(n, dtype=torch.float32, device=self._dev)
            call("rs_din_prepare", ptr(self.kernels[0]), ptr(self.biases[0]), ptr(self.alphas[0]), h1,
                 ptr(self.kernels[1]), ptr(self.biases[1]), ptr(self.alphas[1]), h2, ptr(self.out_kernel),
                 ptr(self.out_bias), self.T, k, ptr(prep), _stream())
            self._ids_prep, self._ids_key = prep, key
        return self._ids_prep

    def forward_ids(self, table, vocab, hist, cand, err=None, out=None, scores=None, cand_out=None):
        """Attention over key = value = table[hist], query = table[cand],
        mask = hist != 0 (model/din.py:56-80) without materialising [B,T,k].
        ``cand_out`` [B, k] (any row stride): also write the candidate rows
        table[cand] there, in the same launch (DIN.call's concat)."""
        B, T = hist.shape
        k = table.shape[1]
        if self.out_kernel is None:
            self.build(T, k)
        if T != self.T:
            raise ValueError(f"Attention built for T={self.T} (PReLU alpha is [T,h]); got T={T}")
        if out is None:
            out = torch.empty(B, k, dtype=torch.float32, device=self._dev)
        if scores is None:
            scores = torch.empty(B, T, dtype=torch.float32, device=self._dev)
        if scores.numel() < B * T:
            raise ValueError("forward_ids: scores workspace needs B*T elements")
        h1, h2 = self.hidden_units
        if cand_out is not None:
            if cand_out.shape != (B, k) or cand_out.stride(1) != 1 or cand_out.dtype != torch.float32:
                raise ValueError("forward_ids: cand_out must be a float32 [B, k] view with unit column stride")
            call("rs_din_attention_ids_cand_fwd", ptr(hist), _lib.id_kind(hist), hist.stride(0), ptr(cand),
                 cand.stride(0), T, k, ptr(table), vocab, h1, h2, ptr(self.prepared_ids(k)), ptr(scores), ptr(out),
                 out.stride(0), ptr(cand_out), cand_out.stride(0), B, ptr(err), _stream())
            return out
        call("rs_din_attention_ids_fwd", ptr(hist), _lib.id_kind(hist), hist.stride(0), ptr(cand),
             cand.stride(0), T, k, ptr(table), vocab, h1, h2, ptr(self.prepared_ids(k)), ptr(scores), ptr(out),
             out.stride(0), B, ptr(err), _stream())
        return out

    def keras_weights(self):
        out = {}
        for i in range(len(self.kernels)):
            out[f"dense_{i}/kernel"] = self.kernels[i]
            out[f"dense_{i}/bias"] = self.biases[i]
            out[f"dense_{i}/prelu/alpha"] = self.alphas[i]
        for i, d in enumerate(self.dice):
            out.update({f"dice_{i}/{k}": v for k, v in d.keras_weights().items()})
        out["out/kernel"] = self.out_kernel
        out["out/bias"] = self.out_bias
        return out

    def set_keras_weights(self, weights, strict=True):
        own = self.keras_weights()
        with torch.no_grad():
            for name, p in own.items():
                if name in weights:
                    p.copy_(torch.as_tensor(weights[name], dtype=torch.float32).reshape(p.shape))
                elif strict:
                    raise KeyError(name)

    def forward(self, inputs, out=None):
        query, key, value, mask = inputs
        q = _to_device_f32(query, self._dev)
        key = _to_device_f32(key, self._dev)
        value = key if value is None else _to_device_f32(value, self._dev)
        mask = _to_device_f32(mask, self._dev)
        q, key, value, mask = (t.contiguous() for t in (q, key, value, mask))  # the kernels take dense rows
        B, T, k = key.shape
        if self.out_kernel is None:
            self.build(T, k)
        if T != self.T and self.activation == "prelu":
            raise ValueError(f"Attention built for T={self.T} (PReLU alpha is [T,h]); got T={T}")
        if out is None:
            out = torch.empty(B, k, dtype=torch.float32, device=self._dev)
        s = _stream()
        if self.activation == "prelu" and not self.fused_ok(k):
            n = len(self.hidden_units)
            hid = (C.c_int * max(n, 1))(*self.hidden_units)
            wsz = _lib.lib().rs_din_attention_gen_workspace_size(B, T, k, n, hid)
            if wsz < 0:
                _lib.check(-1, "rs_din_attention_gen_workspace_size")
            ws = self.__dict__.get("_gen_ws")
            if ws is None or ws.numel() < wsz:
                ws = self.__dict__["_gen_ws"] = torch.empty(wsz, dtype=torch.uint8, device=self._dev)
            pa = lambda ts: (C.c_void_p * max(n, 1))(*[ptr(t) for t in ts])
            call("rs_din_attention_gen_fwd", ptr(q), ptr(key), ptr(value), ptr(mask), T, k, n, hid, pa(self.kernels), pa(self.biases), pa(self.alphas),
                 ptr(self.out_kernel), ptr(self.out_bias), ptr(out), B, ptr(ws), ws.numel(), s)
        elif self.activation == "prelu":
            h1, h2 = self.hidden_units
            call("rs_din_attention_fwd", ptr(q), ptr(key), ptr(value), ptr(mask), T, k, ptr(self.kernels[0]),
                 ptr(self.biases[0]), ptr(self.alphas[0]), h1, ptr(self.kernels[1]), ptr(self.biases[1]),
                 ptr(self.alphas[1]), h2, ptr(self.out_kernel), ptr(self.out_bias), ptr(out), B, s)
        else:
            nl = len(self.dice)
            if nl:
                al = torch.stack([d.alphas for d in self.dice]).contiguous()
                mu = torch.stack([d.moving_mean for d in self.dice]).contiguous()
                var = torch.stack([d.moving_variance for d in self.dice]).contiguous()
                eps = self.dice[0].epsilon
            else:
                al = mu = var = None
                eps = 1e-9
            call("rs_din_attention_dice_fwd", ptr(q), ptr(key), ptr(value), ptr(mask), T, k, nl, ptr(al), ptr(mu),
                 ptr(var), eps, ptr(self.out_kernel), ptr(self.out_bias), ptr(out), B, s)
        return out


def sigmoid_combine(a, b=None, c0=1.0, c1=1.0, out=None):
    """out = sigmoid(c0*a + c1*b) elementwise (model heads)."""
    if out is None:
        out = torch.empty_like(a)
    call("rs_sigmoid_combine", ptr(a), ptr(b), float(c0), float(c1), ptr(out), a.numel(), _stream())
    return out


# ------------------------------------ other interactions
class InteractionLayer(KerasModule):
    """InteractionLayer() — layer/interaction.py:280-297: [B,F,k] -> [B,P,k]
    element-wise products of the (i<j) row-major field pairs
    (rs_pair_products_fwd)."""

    def __init__(self, device=None):
        super().__init__(device)

    def forward(self, inputs, out=None):
        e = _to_device_f32(inputs, self._dev).contiguous()
        B, F, k = e.shape
        P = F * (F - 1) // 2
        if out is None:
            out = torch.empty(B, P, k, dtype=torch.float32, device=self._dev)
        call("rs_pair_products_fwd", ptr(e), F * k, F, k, B, ptr(out), _stream())
        return out


class AttentionLayer(KerasModule):
    """AttentionLayer() — layer/interaction.py:300-319.  Holds the reference's
    weights (attention_w = Dense(n_rows, relu), attention_h = Dense(1)) for
    Keras-name weight exchange; its softmax runs over a size-1 axis, so every
    score is exactly 1 and the output is the sum over the rows
    (rs_attention_pool_fwd) — the weights cannot change the result."""

    def __init__(self, device=None, seed=None):
        super().__init__(device, seed)
        self.attention_w = self.attention_h = None

    def build(self, n_rows, k):
        self.attention_w = Dense(n_rows, activation="relu", device=self._dev, seed=_subseed(self._gen),
                                 input_dim=k)
        self.attention_h = Dense(1, device=self._dev, seed=_subseed(self._gen), input_dim=n_rows)

    def keras_weights(self):
        if self.attention_w is None:
            return {}
        out = {f"dense/{n}": v for n, v in self.attention_w.keras_weights().items()}
        out.update({f"dense_1/{n}": v for n, v in self.attention_h.keras_weights().items()})
        return out

    def set_keras_weights(self, weights, strict=True):
        self.attention_w.set_keras_weights({n[6:]: v for n, v in weights.items() if n.startswith("dense/")}, strict)
        self.attention_h.set_keras_weights({n[8:]: v for n, v in weights.items() if n.startswith("dense_1/")},
                                           strict)

    def forward(self, inputs, out=None):
        x = _to_device_f32(inputs, self._dev).contiguous()
        B, P, k = x.shape
        if self.attention_w is None:
            self.build(P, k)
        if out is None:
            out = torch.empty(B, k, dtype=torch.float32, device=self._dev)
        call("rs_attention_pool_fwd", ptr(x), P * k, P, k, B, ptr(out), _stream())
        return out


def _subseed(gen):
    return int(torch.randint(0, 2 ** 31, (1,), generator=gen))


_AFM_MODES = {"att": 0, "avg": 1, "max": 2}


class AFMLayer(KerasModule):
    """AFMLayer(feature_columns, mode) — layer/interaction.py:322-351:
    per-field Embedding(feat_onehot_dim, embed_dim) -> InteractionLayer ->
    'avg' mean / 'max' max / attention (== sum) over the pairs -> Dense(1) ->
    sigmoid.  ids -> rows -> pooled pairs -> head in ONE launch
    (rs_embed_pair_pool_fwd); the [B,P,k] pair tensor is never formed."""

    def __init__(self, feature_columns, mode, device=None, seed=None):
        super().__init__(device, seed)
        self.dense_feature_columns, self.sparse_feature_columns = feature_columns
        self.mode = mode
        dims = {int(f["embed_dim"]) for f in self.sparse_feature_columns}
        if len(dims) != 1:
            raise ValueError("AFMLayer: every sparse feature needs the same embed_dim (the pairs are stacked)")
        self.k = dims.pop()
        self.nd = len(self.dense_feature_columns)
        self.embed_layer = EmbedLayer(self.sparse_feature_columns, self.k, device=device, seed=_subseed(self._gen))
        self.interaction_layer = InteractionLayer(device=device)
        F = self.embed_layer.n_fields
        self.attention_layer = None
        if mode == "att":
            self.attention_layer = AttentionLayer(device=device, seed=_subseed(self._gen))
            self.attention_layer.build(F * (F - 1) // 2, self.k)
        self.output_layer = Dense(1, device=device, seed=_subseed(self._gen), input_dim=self.k)
        self._err = _ErrFlag(self._dev)

    def pooled(self, inputs, check_ids=True, n_sigmoid=1):
        """(pooled [B,k], head [B,1] = sigmoid^n_sigmoid(Dense(1)(pooled)))."""
        if isinstance(inputs, (tuple, list)):
            ids = _ids_tensor(inputs[1], self._dev)
        else:
            ids = _to_device_f32(inputs, self._dev)[:, self.nd:]
        B = ids.shape[0]
        e = self.embed_layer
        pooled = torch.empty(B, self.k, dtype=torch.float32, device=self._dev)
        head = torch.empty(B, 1, dtype=torch.float32, device=self._dev)
        call("rs_embed_pair_pool_fwd", ptr(ids), _lib.id_kind(ids), ids.stride(0), ptr(e.table),
             ptr(e.field_offsets), ptr(e.field_vocab), e.n_fields, self.k, _AFM_MODES.get(self.mode, 0), None, 0, 0,
             ptr(pooled), self.k, 0, ptr(self.output_layer.kernel), ptr(self.output_layer.bias), n_sigmoid,
             ptr(head), B, ptr(self._err.t), _stream())
        if check_ids:
            self._err.check("AFMLayer")
        return pooled, head

    def forward(self, inputs, check_ids=True):
        return self.pooled(inputs, check_ids, n_sigmoid=1)[1]


class FFMLayer(KerasModule):
    """FFMLayer(feature_columns, k, w_reg=1e-4, v_reg=1e-4) —
    layer/interaction.py:117-163.  Weights in Keras shapes: w0 (1,), w
    (feature_num, 1), v (feature_num, field_num, k), feature_num = nd +
    sum(feat_onehot_dim), field_num = nd + F.  ``forward(X[B, nd+F])`` on
    label-encoded ids: the one-hot x is never formed — row nd + offset_c + id
    of w and v is gathered (rs_ffm_fwd, one wave per sample)."""

    def __init__(self, feature_columns, k, w_reg=1e-4, v_reg=1e-4, device=None, seed=None):
        super().__init__(device, seed)
        self.dense_feature_columns, self.sparse_feature_columns = feature_columns
        self.k = int(k)
        self.w_reg, self.v_reg = w_reg, v_reg
        self.nd = len(self.dense_feature_columns)
        self.onehot_dims = [int(f["feat_onehot_dim"]) for f in self.sparse_feature_columns]
        self.feature_num = sum(self.onehot_dims) + self.nd
        self.field_num = self.nd + len(self.sparse_feature_columns)
        offs = [0]
        for v in self.onehot_dims[:-1]:
            offs.append(offs[-1] + v)
        dev = self._dev
        self.register_buffer("field_offsets", torch.tensor(offs, dtype=torch.int64, device=dev))
        self.register_buffer("field_vocab", torch.tensor(self.onehot_dims, dtype=torch.int64, device=dev))
        self.w0 = nn.Parameter(torch.zeros(1, device=dev), requires_grad=False)
        self.w = nn.Parameter(_normal((self.feature_num, 1), self._gen, dev), requires_grad=False)
        v = torch.empty(self.feature_num, self.field_num, self.k, dtype=torch.float32, device=dev)
        if v.is_cuda:
            g = torch.Generator(device=v.device)
            g.manual_seed(_subseed(self._gen))
            v.normal_(0.0, 0.05, generator=g)
        else:
            v.normal_(0.0, 0.05, generator=self._gen)
        self.v = nn.Parameter(v, requires_grad=False)
        self._err = _ErrFlag(dev)

    def keras_weights(self):
        return {"w0": self.w0, "w": self.w, "v": self.v}

    def set_keras_weights(self, weights, strict=True):
        with torch.no_grad():
            for name, p in self.keras_weights().items():
                p.copy_(torch.as_tensor(weights[name], dtype=torch.float32).reshape(p.shape))

    def logits(self, inputs, n_sigmoid=0):
        if isinstance(inputs, (tuple, list)):
            dense, ids = _to_device_f32(inputs[0], self._dev), _ids_tensor(inputs[1], self._dev)
        else:
            X = _to_device_f32(inputs, self._dev)
            dense, ids = X[:, :self.nd], X[:, self.nd:]
        B = ids.shape[0]
        out = torch.empty(B, 1, dtype=torch.float32, device=self._dev)
        # tf.one_hot (layer/interaction.py:145-146) maps an out-of-range id to
        # a zero row without an error: the kernel does the same (no check)
        call("rs_ffm_fwd", ptr(ids), _lib.id_kind(ids), ids.stride(0), ptr(dense), dense.stride(0), self.nd,
             ptr(self.v), ptr(self.w), ptr(self.w0), ptr(self.field_offsets), ptr(self.field_vocab),
             len(self.onehot_dims), self.k, n_sigmoid, ptr(out), B, None, _stream())
        return out

    def forward(self, inputs):
        return self.logits(inputs, 0)
