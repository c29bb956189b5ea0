"""GPU parity of every C-ABI kernel against the fp64 oracle (oracle/ctr_oracle.py).

Runs on an MI355X through librs_hip.so (the HIP path is the only path).
Sizes are small enough for the oracle to finish in seconds; edge cases follow
what the reference's semantics allow: batch 1 / ragged tails (B not a multiple
of the 16-sample tile), all id dtypes incl. the packed-float X, ids at 0 and
vocab-1, out-of-range ids, fully masked DIN rows, L=0 CrossNet, F=2 PNN.
"""
import numpy as np
import pytest
import torch

from oracle import ctr_oracle as O
from tests.helpers import assert_rel_close, assert_scaled_close, random_ids

pytestmark = pytest.mark.gpu


def _t(a, dev, dtype=torch.float32):
    return torch.as_tensor(np.asarray(a)).to(dtype).to(dev).contiguous()


def _layout(vocabs, dev):
    offs = np.concatenate([[0], np.cumsum(vocabs)[:-1]]).astype(np.int64)
    return offs, _t(offs, dev, torch.int64), _t(vocabs, dev, torch.int64)


# ------------------------------------------------------------------ gather
@pytest.mark.parametrize("id_dtype", ["i32", "i64", "f32"])
@pytest.mark.parametrize("k,nd,B", [(16, 13, 300), (8, 13, 1), (4, 0, 33), (6, 3, 17)])
def test_embed_gather(gpu, id_dtype, k, nd, B):
    from recommender_system_amd import _lib
    rng = np.random.default_rng(k * 100 + B)
    vocabs = rng.integers(1, 500, size=5).tolist() + [1]
    offs, offs_d, voc_d = _layout(vocabs, gpu)
    table = rng.uniform(-0.05, 0.05, size=(sum(vocabs), k)).astype(np.float32)
    ids = random_ids(rng, B, vocabs)
    ids[0, :] = np.array(vocabs) - 1
    dense = rng.random((B, nd)).astype(np.float32)
    if id_dtype == "f32":
        ids_d = _t(ids, gpu, torch.float32)
    else:
        ids_d = _t(ids, gpu, torch.int32 if id_dtype == "i32" else torch.int64)
    dense_d = _t(dense, gpu) if nd else None
    F = len(vocabs)
    out = torch.full((B, nd + F * k), -7.0, device=gpu)
    err = torch.zeros(1, dtype=torch.int32, device=gpu)
    tab_d = _t(table, gpu)
    _lib.call("rs_embed_gather", ids_d.data_ptr(), _lib.id_kind(ids_d), ids_d.stride(0),
              None if dense_d is None else dense_d.data_ptr(), nd, nd, tab_d.data_ptr(),
              offs_d.data_ptr(), voc_d.data_ptr(), F, k, out.data_ptr(), out.stride(0), B, err.data_ptr(), 0)
    torch.cuda.synchronize()
    tables = [table[o:o + v] for o, v in zip(offs, vocabs)]
    ref = np.concatenate([dense, O.embed_layer(ids, tables, np.float64)], 1)
    np.testing.assert_array_equal(out.cpu().numpy(), ref.astype(np.float32))
    assert err.item() == 0


# ------------------------------------------------------- fused gather + FM
@pytest.mark.parametrize("k,kfm,F,nd,B", [
    (16, 10, 26, 13, 300),   # headline shape (DeepFM, dim 16)
    (8, 10, 26, 13, 65),     # reference default EmbedLayer k=8
    (4, 8, 5, 3, 1),
    (32, 15, 7, 13, 40),
    (16, 16, 26, 13, 50),    # kfm+1 > 16 -> two MFMA column tiles
    (8, 31, 9, 0, 31),
    (64, 4, 3, 5, 20),
    (6, 10, 4, 13, 19),      # k % 4 != 0 -> generic kernel
    (16, 40, 4, 2, 9),       # kfm >= 32 -> generic kernel
])
def test_embed_fm_fused(gpu, k, kfm, F, nd, B):
    from recommender_system_amd import _lib
    rng = np.random.default_rng(7 + k + kfm + F)
    vocabs = rng.integers(2, 300, size=F).tolist()
    offs, offs_d, voc_d = _layout(vocabs, gpu)
    d = nd + F * k
    table = rng.uniform(-0.05, 0.05, size=(sum(vocabs), k)).astype(np.float32)
    w1 = (rng.standard_normal((d, 1)) * 0.05).astype(np.float32)
    v = (rng.standard_normal((d, kfm)) * 0.05).astype(np.float32)
    w0 = np.array([0.0123], np.float32)
    ids = random_ids(rng, B, vocabs).astype(np.int32)
    dense = rng.random((B, nd)).astype(np.float32)
    n = _lib.lib().rs_fm_prepared_size(nd, F, k, kfm)
    prep = torch.empty(n, device=gpu)
    w1_d, v_d, w0_d = _t(w1, gpu), _t(v, gpu), _t(w0, gpu)
    _lib.call("rs_fm_prepare", w1_d.data_ptr(), v_d.data_ptr(), nd, F, k, kfm, prep.data_ptr(), 0)
    ids_d, dense_d, tab_d = _t(ids, gpu, torch.int32), _t(dense, gpu), _t(table, gpu)
    logit = torch.full((B,), 99.0, device=gpu)
    x_out = torch.full((B, d), 99.0, device=gpu)
    err = torch.zeros(1, dtype=torch.int32, device=gpu)
    _lib.call("rs_embed_fm_fwd", ids_d.data_ptr(), 0, ids_d.stride(0), dense_d.data_ptr() if nd else None, nd, nd,
              tab_d.data_ptr(), offs_d.data_ptr(), voc_d.data_ptr(), F, k, prep.data_ptr(), w0_d.data_ptr(),
              kfm, logit.data_ptr(), x_out.data_ptr(), B, err.data_ptr(), 0)
    torch.cuda.synchronize()
    tables = [table[o:o + vv] for o, vv in zip(offs, vocabs)]
    x = np.concatenate([dense, O.embed_layer(ids, tables, np.float64)], 1)
    ref = O.fm_layer(x, w0, w1, v)[:, 0]
    np.testing.assert_array_equal(x_out.cpu().numpy(), x.astype(np.float32))
    assert_scaled_close(logit, ref, what="embed_fm logit")
    assert err.item() == 0


# the rs_embed_fm_fwd kernel variants (RS_OPT_EMBED_FM_KERNEL): 0 = K-split
# MFMA, 1 = VALU/DPP tiles, 2 / 3 = pipelined MFMA tiles (2 / 1 per CU).
# Shapes a variant does not cover fall back to the K-split kernel; the cases
# below include several tiles per workgroup (B past 256 or 512 tiles), ragged
# tails, batch 1, odd F, F at each kernel's limit and every id dtype.
@pytest.fixture
def embed_fm_variant(request, gpu):
    from recommender_system_amd import _lib
    prev = _lib.set_option(_lib.OPT_EMBED_FM_KERNEL, request.param)
    yield request.param
    _lib.set_option(_lib.OPT_EMBED_FM_KERNEL, prev)


@pytest.mark.parametrize("embed_fm_variant", [0, 1, 2, 3], indirect=True)
@pytest.mark.parametrize("k,kfm,F,nd,B,idt", [
    (16, 10, 26, 13, 9000, "i32"),   # headline shape, several tiles per workgroup
    (16, 10, 26, 13, 1, "i64"),
    (16, 10, 27, 13, 300, "f32"),    # odd F
    (16, 8, 30, 32, 2071, "i32"),    # VALU limits: F 30, nd 32
    (16, 10, 32, 13, 77, "i64"),     # MFMA-tile limit F = 32
    (8, 10, 26, 13, 4113, "i32"),    # k = 8 (MFMA tiles KV 2; VALU falls back)
    (16, 16, 20, 5, 130, "i32"),     # two MFMA column tiles
    (16, 10, 5, 0, 33, "i32"),       # no dense block
    (16, 10, 26, 13, 16500, "i32"),  # > 1024 tiles: the 4-wave K-split tiles
    (8, 10, 26, 40, 17001, "i64"),   # 4 waves, k 8, more dense k-steps (10) than waves
    (16, 16, 20, 5, 12000, "f32"),   # 8 waves, two column tiles
])
def test_embed_fm_kernel_variants(gpu, embed_fm_variant, k, kfm, F, nd, B, idt):
    from recommender_system_amd import _lib
    rng = np.random.default_rng(B + F + k + kfm)
    vocabs = rng.integers(2, 3000, size=F).tolist()
    offs, offs_d, voc_d = _layout(vocabs, gpu)
    d = nd + F * k
    table = rng.uniform(-0.05, 0.05, size=(sum(vocabs), k)).astype(np.float32)
    w1 = (rng.standard_normal((d, 1)) * 0.05).astype(np.float32)
    v = (rng.standard_normal((d, kfm)) * 0.05).astype(np.float32)
    w0 = np.array([-0.031], np.float32)
    ids = random_ids(rng, B, vocabs)
    ids[0] = np.asarray(vocabs) - 1
    dense = rng.random((B, nd)).astype(np.float32)
    prep = torch.empty(_lib.lib().rs_fm_prepared_size(nd, F, k, kfm), device=gpu)
    w1_d, v_d, w0_d = _t(w1, gpu), _t(v, gpu), _t(w0, gpu)
    _lib.call("rs_fm_prepare", w1_d.data_ptr(), v_d.data_ptr(), nd, F, k, kfm, prep.data_ptr(), 0)
    kind, dt = {"i32": (0, torch.int32), "i64": (1, torch.int64), "f32": (2, torch.float32)}[idt]
    ids_d, dense_d, tab_d = _t(ids, gpu, dt), _t(dense, gpu), _t(table, gpu)
    logit = torch.full((B,), 99.0, device=gpu)
    err = torch.zeros(1, dtype=torch.int32, device=gpu)

    def run(ids_t):
        _lib.call("rs_embed_fm_fwd", ids_t.data_ptr(), kind, ids_t.stride(0),
                  dense_d.data_ptr() if nd else None, nd, nd, tab_d.data_ptr(), offs_d.data_ptr(),
                  voc_d.data_ptr(), F, k, prep.data_ptr(), w0_d.data_ptr(), kfm, logit.data_ptr(), None, B,
                  err.data_ptr(), 0)
        torch.cuda.synchronize()

    run(ids_d)
    tables = [table[o:o + vv] for o, vv in zip(offs, vocabs)]
    x = np.concatenate([dense, O.embed_layer(ids, tables, np.float64)], 1)
    assert_scaled_close(logit, O.fm_layer(x, w0, w1, v)[:, 0], what=f"embed_fm variant {embed_fm_variant}")
    assert err.item() == 0
    bad = ids.copy()
    bad[B - 1, F - 1] = vocabs[F - 1]  # the last sample's last field: out of range
    run(_t(bad, gpu, dt))
    assert err.item() != 0
    err.zero_()
    bad[B - 1, F - 1] = 0
    bad[B // 2, 0] = -1
    run(_t(bad, gpu, dt))
    assert err.item() != 0


@pytest.mark.parametrize("k,kfm,F,nd,B,idt,with_x", [
    (16, 10, 26, 13, 4096, "i32", False),   # the headline: kernarg-metadata kernel
    (16, 10, 26, 13, 8192, "i64", True),    # two tiles per CU, x emitted
    (16, 10, 32, 13, 300, "f32", False),    # F at the kernarg limit
    (8, 10, 26, 40, 1000, "i32", True),     # k 8, more dense k-steps than fit one per wave
    (16, 16, 20, 5, 130, "i32", False),     # two MFMA column tiles
    (16, 10, 26, 13, 9000, "i32", False),   # > 512 tiles: the device-metadata kernel
    (16, 10, 33, 13, 64, "i32", False),     # F > 32: the device-metadata kernel
    (16, 10, 26, 13, 4093, "i64", True),    # ragged last tile, x emitted
    (16, 10, 17, 0, 50, "f32", False),      # no dense block, one pass + a partial pass
    (16, 10, 9, 2, 333, "i32", False),      # fewer fields than waves, one dense k-step
])
def test_embed_fm_host_meta(gpu, k, kfm, F, nd, B, idt, with_x):
    """rs_embed_fm_fwd_hm (field metadata also as kernel arguments, per-wave
    id loads, no id tile) == rs_embed_fm_fwd bit for bit (logit and x) and ==
    the oracle; an out-of-range id sets the flag.  (F < 16 with a dense block:
    the dense k-step belongs to a wave with no field.)"""
    import ctypes as C
    from recommender_system_amd import _lib
    rng = np.random.default_rng(B * 7 + F)
    vocabs = rng.integers(2, 5000, size=F).tolist()
    offs, offs_d, voc_d = _layout(vocabs, gpu)
    hoff = (C.c_int64 * F)(*offs)
    hvoc = (C.c_int64 * F)(*vocabs)
    d = nd + F * k
    table = rng.uniform(-0.05, 0.05, size=(sum(vocabs), k)).astype(np.float32)
    w1 = (rng.standard_normal((d, 1)) * 0.05).astype(np.float32)
    v = (rng.standard_normal((d, kfm)) * 0.05).astype(np.float32)
    w0 = np.array([0.017], np.float32)
    ids = random_ids(rng, B, vocabs)
    ids[0] = np.asarray(vocabs) - 1
    dense = rng.random((B, nd)).astype(np.float32)
    prep = torch.empty(_lib.lib().rs_fm_prepared_size(nd, F, k, kfm), device=gpu)
    w1_d, v_d, w0_d = _t(w1, gpu), _t(v, gpu), _t(w0, gpu)
    _lib.call("rs_fm_prepare", w1_d.data_ptr(), v_d.data_ptr(), nd, F, k, kfm, prep.data_ptr(), 0)
    kind, dt = {"i32": (0, torch.int32), "i64": (1, torch.int64), "f32": (2, torch.float32)}[idt]
    dense_d, tab_d = _t(dense, gpu), _t(table, gpu)
    err = torch.zeros(1, dtype=torch.int32, device=gpu)

    def run(ids_np, hm):
        ids_t = _t(ids_np, gpu, dt)
        logit = torch.full((B,), 99.0, device=gpu)
        x = torch.full((B, d), 7.0, device=gpu) if with_x else None
        common = [ids_t.data_ptr(), kind, ids_t.stride(0), dense_d.data_ptr() if nd else None, nd, nd,
                  tab_d.data_ptr(), offs_d.data_ptr(), voc_d.data_ptr()]
        tail = [F, k, prep.data_ptr(), w0_d.data_ptr(), kfm, logit.data_ptr(), None if x is None else x.data_ptr(), B,
                err.data_ptr(), 0]
        if hm:
            _lib.call("rs_embed_fm_fwd_hm", *common, C.addressof(hoff), C.addressof(hvoc), *tail)
        else:
            _lib.call("rs_embed_fm_fwd", *common, *tail)
        torch.cuda.synchronize()
        return logit, x

    ref_logit, ref_x = run(ids, False)
    assert err.item() == 0
    got_logit, got_x = run(ids, True)
    assert err.item() == 0
    assert torch.equal(got_logit, ref_logit)
    if with_x:
        assert torch.equal(got_x, ref_x)
    tables = [table[o:o + vv] for o, vv in zip(offs, vocabs)]
    x64 = np.concatenate([dense, O.embed_layer(ids, tables, np.float64)], 1)
    assert_scaled_close(got_logit, O.fm_layer(x64, w0, w1, v)[:, 0], what="embed_fm host meta")
    bad = ids.copy()
    bad[B - 1, F - 1] = vocabs[F - 1]
    run(bad, True)
    assert err.item() != 0
    err.zero_()
    bad = ids.copy()
    bad[B // 2, 0] = -1
    run(bad, True)
    assert err.item() != 0


def test_embed_fm_packed_float_X_and_oor(gpu):
    """Packed X[B,39] float ids (Keras int32 truncation) and the OOR flag."""
    from recommender_system_amd import DeepFM
    from tests.helpers import criteo_columns
    rng = np.random.default_rng(3)
    vocabs = rng.integers(2, 200, size=26)
    cols = criteo_columns(vocabs)
    m = DeepFM(cols, 10, 1e-4, 1e-4, [32, 16], 1, "relu", embed_dim=16, seed=1)
    ids = random_ids(rng, 70, vocabs)
    dense = rng.random((70, 13))
    X = np.concatenate([dense, ids + 0.25], 1)  # fractional ids truncate
    a = m.fm_logit(X).cpu().numpy()
    b = m.fm_logit((dense, ids)).cpu().numpy()
    np.testing.assert_array_equal(a, b)
    X[5, 13 + 3] = vocabs[3]  # == vocab -> out of range
    with pytest.raises(IndexError):
        m.fm_logit(X)
    X[5, 13 + 3] = -1.0
    with pytest.raises(IndexError):
        m.fm_logit(X)
    X[5, 13 + 3] = -0.5  # truncates to 0: valid in Keras
    m.fm_logit(X)


# ------------------------------------------------------------- FMLayer dense
@pytest.mark.parametrize("n,kfm,B", [(429, 10, 257), (43, 8, 5), (5000, 8, 33), (7, 20, 16)])
def test_fm_layer_dense(gpu, n, kfm, B):
    from recommender_system_amd import FMLayer
    rng = np.random.default_rng(n)
    x = rng.random((B, n)).astype(np.float32)
    layer = FMLayer(kfm, seed=5)
    y = layer(x)
    w = {k: p.detach().cpu().numpy() for k, p in layer.keras_weights().items()}
    ref = O.fm_layer(x, w["w0"], w["w1"], w["v"])
    assert_scaled_close(y, ref, what="FMLayer")


def test_fm_model_onehot(gpu):
    """FM model: dense one-hot input == compact gather input == oracle."""
    from recommender_system_amd import FM
    rng = np.random.default_rng(11)
    vocabs = rng.integers(2, 60, size=26)
    offs = np.concatenate([[0], np.cumsum(vocabs)[:-1]])
    B, nd = 48, 13
    ids = random_ids(rng, B, vocabs)
    dense = rng.random((B, nd))
    n = nd + int(vocabs.sum())
    onehot = np.zeros((B, n))
    onehot[:, :nd] = dense
    onehot[np.arange(B)[:, None], nd + offs[None, :] + ids] = 1.0
    m = FM(8, seed=2)
    y_dense = m(onehot).cpu().numpy()
    y_gather = m.forward_onehot(dense, ids, offs, vocabs).cpu().numpy()
    p = {k: v.detach().cpu().numpy() for k, v in m.fm.keras_weights().items()}
    ref = O.fm_model(onehot, p)
    assert_rel_close(y_dense, ref, what="FM dense")
    assert_rel_close(y_gather, ref, what="FM gather")


# ---------------------------------------------------------------- CrossNet
@pytest.mark.parametrize("d,L,B", [(429, 3, 300), (221, 6, 17), (37, 1, 1), (64, 0, 20), (429, 20, 33)])
def test_cross_layer(gpu, d, L, B):
    from recommender_system_amd import CrossLayer
    rng = np.random.default_rng(d + L)
    x = (rng.standard_normal((B, d)) * 0.3).astype(np.float32)
    layer = CrossLayer(L, seed=3)
    y = layer(x)
    ws = [w.detach().cpu().numpy() for w in layer.cross_weight]
    bs = [b.detach().cpu().numpy() for b in layer.cross_bias]
    ref = O.cross_layer(x, ws, bs)
    assert_scaled_close(y, ref, what="CrossLayer")


def test_cross_layer_strided_out(gpu):
    from recommender_system_amd import CrossLayer
    rng = np.random.default_rng(1)
    x = (rng.standard_normal((50, 429)) * 0.3).astype(np.float32)
    layer = CrossLayer(3, seed=3)
    z = torch.zeros(50, 431, device=gpu)
    layer(x, out=z[:, 1:430])
    ws = [w.detach().cpu().numpy() for w in layer.cross_weight]
    bs = [b.detach().cpu().numpy() for b in layer.cross_bias]
    assert_scaled_close(z[:, 1:430], O.cross_layer(x, ws, bs), what="CrossLayer strided")
    assert float(z[:, 0].abs().max()) == 0.0 and float(z[:, 430].abs().max()) == 0.0


# ----------------------------------------------------------- inner product
@pytest.mark.parametrize("F,k,B", [(26, 16, 100), (26, 8, 3), (2, 4, 10), (3, 5, 7), (39, 32, 9)])
def test_inner_product(gpu, F, k, B):
    from recommender_system_amd import InnerProductLayer
    rng = np.random.default_rng(F * k)
    e = rng.standard_normal((B, F, k)).astype(np.float32)
    y = InnerProductLayer()(e)
    assert_scaled_close(y, O.inner_product_layer(e), what="InnerProduct")


def test_embed_inner_fused(gpu):
    from recommender_system_amd import PNN
    from tests.helpers import criteo_columns, dnn_params, tables_of
    rng = np.random.default_rng(5)
    vocabs = rng.integers(2, 300, size=26)
    m = PNN(criteo_columns(vocabs), "inner", [64, 32], 1, embed_dim=16, seed=4)
    ids = random_ids(rng, 77, vocabs)
    X = np.concatenate([rng.random((77, 13)), ids], 1)
    z = m.product_inputs(X).cpu().numpy()
    y = m(X)
    hidden, out = dnn_params(m.dnn_layer)
    ref, ref_z = O.pnn_inner(X, {"tables": tables_of(m.embed_layer), "dnn_hidden": hidden, "dnn_out": out})
    assert_scaled_close(z, ref_z, what="PNN inputs")
    assert_scaled_close(y, ref, what="PNN logit")


# -------------------------------------------------------------- DIN attention
def _att_params(layer):
    p = {}
    if layer.activation == "prelu":
        p["prelu"] = [(layer.kernels[i].detach().cpu().numpy(), layer.biases[i].detach().cpu().numpy(),
                       layer.alphas[i].detach().cpu().numpy()) for i in range(len(layer.kernels))]
    else:
        p["dice"] = [(d.alphas.detach().cpu().numpy(), d.moving_mean.detach().cpu().numpy(),
                      d.moving_variance.detach().cpu().numpy(), d.epsilon) for d in layer.dice]
    p["out"] = (layer.out_kernel.detach().cpu().numpy(), layer.out_bias.detach().cpu().numpy())
    return p


@pytest.mark.parametrize("T,k,h,B", [(100, 8, (80, 40), 37), (10, 8, (80, 40), 5), (1, 4, (16, 16), 3),
                                     (33, 16, (128, 100), 9), (20, 32, (64, 8), 4)])
def test_din_attention_prelu(gpu, T, k, h, B):
    from recommender_system_amd import Attention
    rng = np.random.default_rng(T * k)
    q = rng.standard_normal((B, k)).astype(np.float32)
    key = rng.standard_normal((B, T, k)).astype(np.float32)
    lens = rng.integers(0, T + 1, size=B)
    lens[0] = 0  # fully masked row -> uniform average
    mask = (np.arange(T)[None, :] < lens[:, None]).astype(np.float32)
    layer = Attention(h, "prelu", seed=9)
    layer.build(T, k)
    with torch.no_grad():  # non-zero PReLU alphas and biases to exercise them
        for a in layer.alphas:
            a.copy_(torch.as_tensor(rng.uniform(-0.5, 0.5, size=tuple(a.shape)), dtype=torch.float32))
        for b in layer.biases:
            b.copy_(torch.as_tensor(rng.uniform(-0.1, 0.1, size=tuple(b.shape)), dtype=torch.float32))
    y = layer([q, key, key, mask])
    ref = O.attention(q, key, key, mask, _att_params(layer), "prelu")
    assert_scaled_close(y, ref, what="Attention prelu")
    np.testing.assert_allclose(y.cpu().numpy()[0], key[0].mean(0), rtol=1e-5, atol=1e-6)


def test_din_attention_dice(gpu):
    from recommender_system_amd import Attention
    rng = np.random.default_rng(2)
    B, T, k = 11, 50, 8
    q = rng.standard_normal((B, k)).astype(np.float32)
    key = rng.standard_normal((B, T, k)).astype(np.float32)
    mask = (rng.random((B, T)) > 0.3).astype(np.float32)
    layer = Attention((80, 40), "dice", seed=1)
    layer.build(T, k)
    with torch.no_grad():
        for d in layer.dice:
            d.alphas.uniform_(-0.5, 0.5)
            d.moving_mean.uniform_(-0.1, 0.1)
            d.moving_variance.uniform_(0.5, 1.5)
    y = layer([q, key, key, mask])
    assert_scaled_close(y, O.attention(q, key, key, mask, _att_params(layer), "dice"), what="Attention dice")


# ---------------------------------------------------------------- Dense GEMM
@pytest.mark.parametrize("M,K,N,act", [(4096, 429, 256, "relu"), (70, 13, 65, None), (33, 256, 128, "prelu"),
                                       (5, 64, 1, None), (100, 66, 3, "sigmoid"), (1, 1, 7, "relu")])
def test_dense(gpu, M, K, N, act):
    from recommender_system_amd import Dense
    rng = np.random.default_rng(M + K + N)
    x = rng.standard_normal((M, K)).astype(np.float32)
    layer = Dense(N, act, seed=2)
    layer.build(K)
    if act == "prelu":
        with torch.no_grad():
            layer.alpha.uniform_(-0.5, 0.5)
            layer.bias.uniform_(-0.1, 0.1)
    y = layer(x)
    ref = O.dense(x, layer.kernel.cpu().numpy(), layer.bias.cpu().numpy(), act,
                  None if layer.alpha is None else layer.alpha.cpu().numpy())
    assert_scaled_close(y, ref, what=f"Dense {act}")


def test_dice_2d_and_bn(gpu):
    from recommender_system_amd import BatchNormalization, Dice
    rng = np.random.default_rng(8)
    x = rng.standard_normal((40, 66)).astype(np.float32)
    dice = Dice()
    dice.build(66)
    bn = BatchNormalization()
    bn.build(66)
    with torch.no_grad():
        dice.alphas.uniform_(-1, 1)
        dice.moving_mean.uniform_(-0.2, 0.2)
        dice.moving_variance.uniform_(0.5, 2.0)
        for p in (bn.gamma, bn.moving_variance):
            p.uniform_(0.5, 1.5)
        for p in (bn.beta, bn.moving_mean):
            p.uniform_(-0.2, 0.2)
    xd = torch.as_tensor(x, device=gpu)
    yd = dice(xd)
    yb = bn(xd)
    c = lambda t: t.detach().cpu().numpy()
    assert_scaled_close(yd, O.dice(x, c(dice.alphas), c(dice.moving_mean), c(dice.moving_variance), 1e-9), what="Dice")
    assert_scaled_close(yb, O.batchnorm_inference(x, c(bn.moving_mean), c(bn.moving_variance), c(bn.gamma),
                                                  c(bn.beta), 1e-3), what="BN")


# ------------------------------------------------------- fused MLP tower (mlp.hip)
def _tower_ref(x, layers):
    for l in layers:
        x = O.dense(x, l.kernel.cpu().numpy(), l.bias.cpu().numpy(), l.activation,
                    None if l.alpha is None else l.alpha.cpu().numpy())
    return x


# the fused towers' k-group contraction (RS_OPT_MLP_UNROLL): 0 = looped,
# 1 = fully unrolled for the common layer widths (27 / 16 / 8 / 4 / 1 groups)
@pytest.fixture(params=[0, 1])
def mlp_unroll(request, gpu):
    from recommender_system_amd import _lib
    prev = _lib.set_option(_lib.OPT_MLP_UNROLL, request.param)
    yield request.param
    _lib.set_option(_lib.OPT_MLP_UNROLL, prev)


@pytest.mark.parametrize("M,K,hidden,out,act", [(4096, 429, [256, 128, 64], 1, "relu"),
                                                (1000, 741, [256, 128, 64], 1, "relu"),
                                                (37, 37, [50, 3], 7, "prelu"),
                                                (1, 1024, [1024], 16, "relu"),
                                                (130, 20, [16, 16, 16, 16, 16, 16, 16], 2, "sigmoid")])
def test_dnn_tower(gpu, mlp_unroll, M, K, hidden, out, act):
    from recommender_system_amd import DNNLayer
    rng = np.random.default_rng(M + K)
    x = torch.tensor(rng.standard_normal((M, K)).astype(np.float32), device="cuda")
    dnn = DNNLayer(hidden, out, act, seed=5)
    dnn.build(K)
    with torch.no_grad():
        for l in dnn._layers():
            l.bias.uniform_(-0.1, 0.1)
            if l.alpha is not None:
                l.alpha.uniform_(-0.5, 0.5)
    assert dnn.tower_ok()
    y = dnn(x)
    torch.cuda.synchronize()
    assert_scaled_close(y, _tower_ref(x.cpu().numpy(), dnn._layers()), what=f"DNN tower {hidden}")
    # the per-layer Dense path agrees with the fused tower
    h = x
    for l in dnn._layers():
        h = l(h)
    assert_scaled_close(y, h, what="tower vs per-layer")


def test_dnn_tower_head_strided_and_permuted(gpu):
    """head=1 (DeepFM sigmoid(0.5 fm + 0.5 dnn)), a strided input/output view
    and an LDS column permutation (in_rows) give the same numbers."""
    from recommender_system_amd import DNNLayer
    rng = np.random.default_rng(3)
    M, K = 300, 45
    big = torch.tensor(rng.standard_normal((M, K + 7)).astype(np.float32), device="cuda")
    x = big[:, 3:3 + K]
    dnn = DNNLayer([64, 32], 1, "relu", seed=9)
    dnn.build(K)
    fm = torch.tensor(rng.standard_normal((M, 1)).astype(np.float32), device="cuda")
    y = dnn.tower(x, extra=fm, c0=0.5, c1=0.5, head=True)
    z = _tower_ref(x.cpu().numpy(), dnn._layers())
    ref = 1.0 / (1.0 + np.exp(-(0.5 * z + 0.5 * fm.cpu().numpy().astype(np.float64))))
    assert_rel_close(y, ref, what="tower head")
    out = torch.zeros(M, 5, device="cuda")
    dnn.tower(x, out=out[:, 2:3])
    assert_scaled_close(out[:, 2:3], z, what="tower strided out")
    assert float(out[:, :2].abs().sum() + out[:, 3:].abs().sum()) == 0.0
    # permuted LDS columns: column p of the staged tile holds Keras row perm[p]
    perm = rng.permutation(K)
    Kp = (K + 15) // 16 * 16
    in_rows = torch.full((Kp,), -1, dtype=torch.int32, device="cuda")
    in_rows[:K] = torch.tensor(perm, dtype=torch.int32)
    prep = dnn.prepared(in_rows)
    from recommender_system_amd import _lib
    import ctypes as C
    dims = dnn._dims()
    n = len(dims) - 1
    xp = x[:, torch.tensor(perm, device="cuda")].contiguous()
    y2 = torch.empty(M, 1, device="cuda")
    _lib.call("rs_mlp_fwd", xp.data_ptr(), xp.stride(0), n, (C.c_int * (n + 1))(*dims),
              (C.c_int * n)(*[_lib.ACT[l.activation] for l in dnn._layers()]), prep.data_ptr(), y2.data_ptr(), 1,
              0, None, 1.0, 1.0, M, _lib.stream())
    assert_scaled_close(y2, z, what="tower permuted input")


# ----------------------------------------------- fused DeepFM (rs_deepfm_fwd)
@pytest.mark.parametrize("k,B,id_dtype,hidden", [(16, 4096, np.int32, [256, 128, 64]), (8, 1000, np.int64, [256, 128, 64]),
                                                 (16, 33, np.int32, [40, 24]), (8, 1, np.int64, [16])])
def test_deepfm_fused(gpu, mlp_unroll, k, B, id_dtype, hidden):
    """One-launch DeepFM == two-launch path == fp64 oracle; the optional FM
    logit output matches the standalone FM kernel."""
    from recommender_system_amd import DeepFM
    from tests.helpers import criteo_columns, dnn_params, tables_of
    rng = np.random.default_rng(k + B)
    vocabs = rng.integers(2, 5000, size=26)
    m = DeepFM(criteo_columns(vocabs, embed_dim=k), 10, 1e-4, 1e-4, hidden, 1, "relu", embed_dim=k, seed=7)
    with torch.no_grad():
        for l in m.dnn._layers():
            l.bias.uniform_(-0.1, 0.1)
    assert m.fused_ok()
    ids = random_ids(rng, B, vocabs, id_dtype)
    dense = rng.random((B, 13)).astype(np.float32)
    fm = torch.empty(B, 1, device="cuda")
    y = m.forward_fused((dense, ids), fm_logit=fm)
    y2 = m.forward_unfused((dense, ids))
    torch.cuda.synchronize()
    hidden_p, out_p = dnn_params(m.dnn)
    p = {"tables": tables_of(m.embed_layer), "w0": m.fm.w0.cpu().numpy(), "w1": m.fm.w1.cpu().numpy(),
         "v": m.fm.v.cpu().numpy(), "dnn_hidden": hidden_p, "dnn_out": out_p}
    ref, ref_fm, _ = O.deepfm(None, p, inputs=(dense, ids))
    assert_rel_close(y, ref, what="fused DeepFM")
    assert_rel_close(y2, ref, what="unfused DeepFM")
    assert_scaled_close(fm, ref_fm, what="fused DeepFM fm logit")


def test_deepfm_fused_oor_and_float_ids(gpu):
    from recommender_system_amd import DeepFM
    from tests.helpers import criteo_columns
    rng = np.random.default_rng(11)
    vocabs = rng.integers(2, 300, size=26)
    m = DeepFM(criteo_columns(vocabs, embed_dim=16), 10, 1e-4, 1e-4, [64, 32], 1, "relu", embed_dim=16, seed=2)
    ids = random_ids(rng, 50, vocabs)
    dense = rng.random((50, 13))
    X = np.concatenate([dense, ids + 0.5], 1)
    a = m(X).cpu().numpy()
    b = m((dense, ids)).cpu().numpy()
    np.testing.assert_array_equal(a, b)
    X[7, 13 + 9] = vocabs[9]
    with pytest.raises(IndexError):
        m(X)


# ------------------------------------------- fused DCN input + CrossNet
@pytest.mark.parametrize("form", [0, 1])
@pytest.mark.parametrize("k,L,B,id_dtype", [(16, 3, 4096, np.int32), (8, 2, 37, np.int64), (4, 1, 5, np.int32),
                                            (16, 20, 100, np.int64), (8, 0, 9, np.int32), (16, 3, 4093, np.int64),
                                            (16, 16, 33, np.float32), (16, 1, 1, np.int32)])
def test_embed_cross_fused(gpu, form, k, L, B, id_dtype):
    """embed + CrossNet (rs_embed_cross_fwd[_hm]) vs the fp64 oracle; at k 16
    both RS_OPT_CROSS_KERNEL forms of the kernarg front end (0: contraction
    from the gathered registers, 1: staged-tile contraction)."""
    from recommender_system_amd import DCN, _lib
    from tests.helpers import criteo_columns, tables_of
    prev = _lib.set_option(_lib.OPT_CROSS_KERNEL, form)
    try:
        _embed_cross_case(k, L, B, id_dtype)
    finally:
        _lib.set_option(_lib.OPT_CROSS_KERNEL, prev)


def _embed_cross_case(k, L, B, id_dtype):
    from recommender_system_amd import DCN
    from tests.helpers import criteo_columns, tables_of
    rng = np.random.default_rng(k * 7 + L)
    vocabs = rng.integers(2, 3000, size=26)
    m = DCN(criteo_columns(vocabs, embed_dim=k), [32], 1, "relu", layer_num=L, embed_dim=k, seed=3)
    with torch.no_grad():
        for b in m.cross_layer.cross_bias:
            b.uniform_(-0.1, 0.1)
    ids = random_ids(rng, B, vocabs, id_dtype)
    dense = rng.random((B, 13)).astype(np.float32)
    out = torch.full((B, m.d + 3), 7.0, device="cuda")
    y = m.cross_fused((dense, ids), out=out[:, :m.d])
    torch.cuda.synchronize()
    x0 = np.concatenate([dense.astype(np.float64), O.embed_layer(ids, tables_of(m.embed_layer))], 1)
    ws = [w.cpu().numpy() for w in m.cross_layer.cross_weight]
    bs = [b.cpu().numpy() for b in m.cross_layer.cross_bias]
    assert_scaled_close(y, O.cross_layer(x0, ws, bs), what=f"embed+cross L={L}")
    assert float((out[:, m.d:] - 7.0).abs().max()) == 0.0
    bad = ids.copy()
    bad[B // 2, 4] = vocabs[4]
    with pytest.raises(IndexError):
        m.cross_fused((dense, bad))


# ------------------------------------- DIN attention from ids (rs_din_attention_ids_fwd)
@pytest.mark.parametrize("form", [0, 1])
@pytest.mark.parametrize("T,k,h,B,id_dtype", [(100, 8, (80, 40), 2048, np.int64), (10, 8, (80, 40), 5, np.int32),
                                              (1, 4, (16, 16), 3, np.int64), (33, 16, (128, 64), 21, np.int32),
                                              (17, 8, (20, 7), 40, np.int32), (37, 4, (80, 40), 13, np.int32),
                                              (150, 16, (80, 40), 9, np.int64), (100, 8, (80, 40), 2045, np.int32),
                                              (100, 16, (80, 40), 70, np.int64), (128, 4, (80, 40), 17, np.int32)])
def test_din_attention_ids(gpu, form, T, k, h, B, id_dtype):
    """keys = values = table[hist], query = table[cand], mask = hist != 0;
    padded positions keep their (id 0) rows in the pooled values, a fully
    padded row averages them uniformly — as the reference.  form 0 = the
    one-launch kernel (din_fused, the reference's (80, 40) widths), 1 = the
    two-launch scores + pool path (RS_OPT_DIN_KERNEL)."""
    from recommender_system_amd import Attention, _lib
    prev = _lib.set_option(_lib.OPT_DIN_KERNEL, form)
    try:
        _din_ids_case(T, k, h, B, id_dtype)
    finally:
        _lib.set_option(_lib.OPT_DIN_KERNEL, prev)


def _din_ids_case(T, k, h, B, id_dtype):
    from recommender_system_amd import Attention
    rng = np.random.default_rng(T * k + B)
    V = 5000
    table_np = rng.standard_normal((V, k)).astype(np.float32)
    lens = rng.integers(0, T + 1, size=B)
    lens[0] = 0
    hist = rng.integers(1, V, size=(B, T))
    hist = np.where(np.arange(T)[None, :] < lens[:, None], hist, 0).astype(id_dtype)
    cand = rng.integers(0, V, size=(B, 1)).astype(id_dtype)
    layer = Attention(h, "prelu", seed=4)
    layer.build(T, k)
    with torch.no_grad():
        for a in layer.alphas:
            a.copy_(torch.as_tensor(rng.uniform(-0.5, 0.5, size=tuple(a.shape)), dtype=torch.float32))
        for b in layer.biases:
            b.copy_(torch.as_tensor(rng.uniform(-0.1, 0.1, size=tuple(b.shape)), dtype=torch.float32))
    assert layer.ids_ok(k)
    table = torch.tensor(table_np, device="cuda")
    err = torch.zeros(1, dtype=torch.int32, device="cuda")
    y = layer.forward_ids(table, V, torch.tensor(hist, device="cuda"), torch.tensor(cand, device="cuda"), err=err)
    torch.cuda.synchronize()
    key = table_np[hist]
    q = table_np[cand[:, 0]]
    mask = (hist != 0).astype(np.float32)
    ref = O.attention(q, key, key, mask, _att_params(layer), "prelu")
    assert_scaled_close(y, ref, what="DIN attention from ids")
    assert err.item() == 0
    # the same launch also copies the candidate rows (DIN.call's concat: a
    # strided [B, k] view): the pool unchanged bit for bit, the copy exact
    emb = torch.full((B, 3 * k + 1), 7.0, device="cuda")
    y2 = layer.forward_ids(table, V, torch.tensor(hist, device="cuda"), torch.tensor(cand, device="cuda"), err=err,
                           out=emb[:, :k], cand_out=emb[:, k:2 * k])
    torch.cuda.synchronize()
    assert torch.equal(y2, y)
    assert np.array_equal(emb[:, k:2 * k].cpu().numpy(), q)
    assert bool((emb[:, 2 * k:] == 7.0).all())
    bad_c = cand.copy()
    bad_c[B // 2, 0] = V
    layer.forward_ids(table, V, torch.tensor(hist, device="cuda"), torch.tensor(bad_c, device="cuda"), err=err,
                      out=emb[:, :k], cand_out=emb[:, k:2 * k])
    torch.cuda.synchronize()
    assert err.item() != 0 and bool((emb[B // 2, k:2 * k] == 0).all())
    err.zero_()
    bad = hist.copy()
    bad[B - 1, 0] = V
    layer.forward_ids(table, V, torch.tensor(bad, device="cuda"), torch.tensor(cand, device="cuda"), err=err)
    torch.cuda.synchronize()
    assert err.item() != 0


# ------------------------------------------------------------ empty batches
def test_empty_batches_every_path(gpu):
    """B = 0 through every C-ABI path: no launch, no error, empty outputs."""
    from recommender_system_amd import DCN, DeepFM, DNNLayer, FM, PNN, Attention, InnerProductLayer
    from tests.helpers import criteo_columns
    vocabs = [30] * 26
    cols = criteo_columns(vocabs, embed_dim=16)
    ids = np.zeros((0, 26), np.int32)
    dense = np.zeros((0, 13), np.float32)
    m = DeepFM(cols, 10, 1e-4, 1e-4, [32, 16], 1, "relu", embed_dim=16, seed=1)
    assert m((dense, ids)).shape == (0, 1)
    assert m.forward_unfused((dense, ids)).shape == (0, 1)
    assert m.fm_logit((dense, ids)).shape == (0, 1)
    d = DCN(cols, [32], 1, "relu", layer_num=2, embed_dim=16, seed=1)
    assert d((dense, ids)).shape == (0, 1)
    assert d.cross_fused((dense, ids)).shape == (0, 13 + 26 * 16)
    p = PNN(cols, "inner", [32], 1, embed_dim=16, seed=1)
    assert p((dense, ids)).shape == (0, 1)
    dnn = DNNLayer([32], 1, "relu", seed=1)
    dnn.build(20)
    assert dnn(torch.zeros(0, 20, device="cuda")).shape == (0, 1)
    ip = InnerProductLayer()
    assert ip(torch.zeros(0, 5, 8, device="cuda")).shape == (0, 10)
    att = Attention((16, 8), "prelu", seed=1)
    att.build(7, 8)
    table = torch.randn(50, 8, device="cuda")
    out = att.forward_ids(table, 50, torch.zeros(0, 7, dtype=torch.int32, device="cuda"),
                          torch.zeros(0, 1, dtype=torch.int32, device="cuda"))
    assert out.shape == (0, 8)
    fm = FM(8, 1e-4, 1e-4, seed=1)
    assert fm(np.zeros((0, 43), np.float32)).shape == (0, 1)


# ---------------------------------------------------- PNN outer / both modes
@pytest.mark.parametrize("F,k,B", [(26, 16, 100), (26, 8, 3), (2, 4, 10), (39, 32, 9), (9, 64, 17)])
def test_outer_product(gpu, F, k, B):
    from recommender_system_amd import OuterProductLayer
    rng = np.random.default_rng(F * k + B)
    e = rng.standard_normal((B, F, k)).astype(np.float32)
    layer = OuterProductLayer(seed=3)
    y = layer(e)
    ref = O.outer_product_layer(e, layer.W.cpu().numpy())
    assert_scaled_close(y, ref, what=f"OuterProduct F={F} k={k}")


@pytest.mark.parametrize("mode,k,B,id_dtype", [("outer", 16, 4096, np.int32), ("both", 16, 37, np.int64),
                                               ("both", 8, 5, np.int32), ("outer", 4, 64, np.int64)])
def test_pnn_modes_fused(gpu, mode, k, B, id_dtype):
    from recommender_system_amd import PNN
    from tests.helpers import criteo_columns, dnn_params, tables_of
    rng = np.random.default_rng(B + k)
    vocabs = rng.integers(2, 4000, size=26)
    m = PNN(criteo_columns(vocabs, embed_dim=k), mode, [64, 32], 1, embed_dim=k, seed=5)
    ids = random_ids(rng, B, vocabs, id_dtype)
    dense = rng.random((B, 13)).astype(np.float32)
    x = m.product_inputs((dense, ids))
    y = m((dense, ids))
    hidden, out = dnn_params(m.dnn_layer)
    p = {"tables": tables_of(m.embed_layer), "outer_W": m.outer_product_layer.W.cpu().numpy(),
         "dnn_hidden": hidden, "dnn_out": out}
    ref_y, ref_x = O.pnn(None, p, mode=mode, inputs=(dense, ids))
    assert_scaled_close(x, ref_x, what=f"PNN {mode} inputs")
    assert_scaled_close(y, ref_y, what=f"PNN {mode} logit")


# ------------------------------------------------- fused DCN (rs_dcn_fwd)
@pytest.mark.parametrize("k,L,hidden,out_dim,B,id_dtype", [(16, 3, [256, 128, 64], 1, 4096, np.int32),
                                                           (8, 2, [40, 24], 3, 37, np.int64),
                                                           (4, 0, [16], 1, 5, np.int32),
                                                           (16, 20, [32], 2, 100, np.int64),
                                                           (16, 3, [48], 1, 333, np.int64),
                                                           (16, 15, [256, 128, 64], 1, 61, np.float32)])
def test_dcn_fused(gpu, mlp_unroll, k, L, hidden, out_dim, B, id_dtype):
    """One-launch DCN == the layer-by-layer path == the fp64 oracle."""
    from recommender_system_amd import DCN
    from tests.helpers import criteo_columns, dnn_params, tables_of
    rng = np.random.default_rng(k + L + B)
    vocabs = rng.integers(2, 3000, size=26)
    m = DCN(criteo_columns(vocabs, embed_dim=k), hidden, out_dim, "relu", layer_num=L, embed_dim=k, seed=6)
    with torch.no_grad():
        for b in m.cross_layer.cross_bias:
            b.uniform_(-0.1, 0.1)
        for l in m.dense_layer._layers():
            l.bias.uniform_(-0.1, 0.1)
        m.output_layer.bias.uniform_(-0.1, 0.1)
    assert m.fused_ok()
    ids = random_ids(rng, B, vocabs, id_dtype)
    dense = rng.random((B, 13)).astype(np.float32)
    y = m.forward_fused((dense, ids))
    y2 = m.forward_unfused((dense, ids))
    torch.cuda.synchronize()
    hidden_p, out_p = dnn_params(m.dense_layer)
    p = {"tables": tables_of(m.embed_layer), "cross_w": [w.cpu().numpy() for w in m.cross_layer.cross_weight],
         "cross_b": [b.cpu().numpy() for b in m.cross_layer.cross_bias], "dnn_hidden": hidden_p, "dnn_out": out_p,
         "out_kernel": m.output_layer.kernel.cpu().numpy(), "out_bias": m.output_layer.bias.cpu().numpy()}
    ref, _ = O.dcn(None, p, inputs=(dense, ids))
    assert_rel_close(y, ref, what="fused DCN")
    assert_rel_close(y2, ref, what="layer-by-layer DCN")
    bad = ids.copy()
    bad[0, 3] = vocabs[3]
    with pytest.raises(IndexError):
        m.forward_fused((dense, bad))


# --------------------------------------- full-size table: 64-bit addressing
def test_full_size_table_addressing(gpu):
    """The headline layout at full size — 26 x 1e7 rows x 16 fp32 = 16.6 GB,
    byte offsets past 2^33 — through DeepFM (fused, FM logit, two-launch),
    DCN (fused, cross) and PNN ('both').  Only the rows the batch touches are
    written (ids drawn near the top of each field's range); the oracle works
    on exactly those rows."""
    from recommender_system_amd import DCN, PNN, DeepFM
    from tests.helpers import criteo_columns, dnn_params
    V, F, k, B = 10_000_000, 26, 16, 64
    vocabs = [V] * F
    rng = np.random.default_rng(99)
    ids = np.stack([rng.integers(V - 1000, V, size=B) for _ in range(F)], 1).astype(np.int64)
    ids[0] = V - 1
    dense = rng.random((B, 13)).astype(np.float32)
    cols = criteo_columns(vocabs, embed_dim=k)
    m = DeepFM(cols, 10, 1e-4, 1e-4, [64, 32], 1, "relu", embed_dim=k, seed=1)
    e = m.embed_layer
    rows = (e.field_offsets.cpu().numpy()[None, :] + ids).reshape(-1)
    assert rows.max() * k * 4 > 2 ** 33
    vals = rng.uniform(-0.05, 0.05, size=(rows.size, k)).astype(np.float32)
    with torch.no_grad():
        e.table[torch.as_tensor(rows, device="cuda")] = torch.as_tensor(vals, device="cuda")
    x_emb = e.table[torch.as_tensor(rows, device="cuda")].cpu().numpy().reshape(B, F * k)  # dup-safe
    x = np.concatenate([dense, x_emb], 1)
    hidden, out = dnn_params(m.dnn)
    fm = O.fm_layer(x, m.fm.w0.cpu().numpy(), m.fm.w1.cpu().numpy(), m.fm.v.cpu().numpy())
    ref = 1.0 / (1.0 + np.exp(-(0.5 * (fm + O.dnn_layer(x, hidden, out)))))
    assert_rel_close(m((dense, ids)), ref, what="DeepFM fused @16.6 GB")
    assert_rel_close(m.forward_unfused((dense, ids)), ref, what="DeepFM two-launch @16.6 GB")
    assert_scaled_close(m.fm_logit((dense, ids)), fm, what="FM logit @16.6 GB")
    d = DCN(cols, [32], 1, "relu", layer_num=2, embed_dim=k, seed=2)
    d.embed_layer.table = e.table  # share the 16.6 GB table
    ws = [w.cpu().numpy() for w in d.cross_layer.cross_weight]
    bs = [b.cpu().numpy() for b in d.cross_layer.cross_bias]
    assert_scaled_close(d.cross_fused((dense, ids)), O.cross_layer(x, ws, bs), what="embed+cross @16.6 GB")
    h2, o2 = dnn_params(d.dense_layer)
    z = np.concatenate([O.cross_layer(x, ws, bs), O.dnn_layer(x, h2, o2)], 1)
    dref = O.dense(z, d.output_layer.kernel.cpu().numpy(), d.output_layer.bias.cpu().numpy(), "sigmoid")
    assert_rel_close(d((dense, ids)), dref, what="DCN fused @16.6 GB")
    p = PNN(cols, "both", [32], 1, embed_dim=k, seed=3)
    p.embed_layer.table = e.table
    xin = p.product_inputs((dense, ids))
    zz = x_emb.reshape(B, F, k)
    pref = np.concatenate([x_emb, O.inner_product_layer(zz), O.outer_product_layer(zz, p.outer_product_layer.W.cpu().numpy())], 1)
    assert_scaled_close(xin, pref, what="PNN both @16.6 GB")


@pytest.mark.parametrize("embed_fm_variant", [0, 1, 2, 3], indirect=True)
def test_headline_shape_full_size(gpu, embed_fm_variant):
    """The headline configuration itself (BASELINE metric: batch 4096, 26 x
    1e7 x 16 fp32 table = 16.6 GB, uniform int32 ids over the full range):
    rs_embed_fm_fwd (the benched kernel, DeepFM.fm_logit) and the fused DeepFM
    forward against the fp64 oracle on the rows the batch touches."""
    from recommender_system_amd import DeepFM
    from tests.helpers import criteo_columns, dnn_params
    V, F, k, B = 10_000_000, 26, 16, 4096
    rng = np.random.default_rng(4096)
    ids = rng.integers(0, V, size=(B, F)).astype(np.int32)
    ids[0] = V - 1
    dense = rng.random((B, 13)).astype(np.float32)
    m = DeepFM(criteo_columns([V] * F, embed_dim=k), 10, 1e-4, 1e-4, [256, 128, 64], 1, "relu", embed_dim=k, seed=5)
    e = m.embed_layer
    rows = torch.as_tensor((e.field_offsets.cpu().numpy()[None, :] + ids).reshape(-1), device="cuda")
    x = np.concatenate([dense, e.table[rows].cpu().numpy().reshape(B, F * k)], 1)
    fm = O.fm_layer(x, m.fm.w0.cpu().numpy(), m.fm.w1.cpu().numpy(), m.fm.v.cpu().numpy())
    assert_scaled_close(m.fm_logit((dense, ids)), fm, what="FM logit, headline shape")
    hidden, out = dnn_params(m.dnn)
    ref = 1.0 / (1.0 + np.exp(-(0.5 * (fm + O.dnn_layer(x, hidden, out)))))
    assert_rel_close(m((dense, ids)), ref, what="DeepFM fused, headline shape")


# ------------- kernel-argument front end of the DCN / PNN kernels (the _hm entries)
@pytest.mark.parametrize("F,B,id_dtype", [(26, 4096, np.int32), (26, 333, np.int64), (20, 17, np.float32),
                                          (32, 1, np.int32), (9, 64, np.int64)])
def test_hm_front_end_bit_identical(gpu, F, B, id_dtype):
    """rs_embed_cross_fwd_hm / rs_dcn_fwd_hm / rs_embed_inner_fwd_hm /
    rs_embed_product_fwd_hm (k = 16: field metadata as kernel arguments, the
    rows gathered by the headline kernel's per-wave front end) write exactly
    what the cooperative-id-tile kernels write (rs_embed_cross_fwd, ...), and
    flag an out-of-range id of a valid sample."""
    import ctypes as C
    from recommender_system_amd import DCN, PNN, _lib
    from tests.helpers import criteo_columns
    rng = np.random.default_rng(F * 1000 + B)
    vocabs = rng.integers(2, 3000, size=F)
    cols = criteo_columns(vocabs, embed_dim=16)
    m = DCN(cols, [64, 32], 1, "relu", layer_num=3, embed_dim=16, seed=2)
    p = PNN(cols, "both", [32], 1, embed_dim=16, seed=3)
    ids_np = random_ids(rng, B, vocabs, np.int64)
    dt = {np.int32: torch.int32, np.int64: torch.int64, np.float32: torch.float32}[id_dtype]
    ids = torch.as_tensor(ids_np, device=gpu).to(dt)
    kind = _lib.id_kind(ids)
    dense = torch.rand(B, 13, device=gpu)
    err = torch.zeros(1, dtype=torch.int32, device=gpu)
    st = _lib.stream()

    def both(entry, args_before, args_after, out):
        outs = []
        for hm in (False, True):
            out.fill_(7.0)
            if hm:
                _lib.call(entry + "_hm", *args_before, *args_hm, *args_after)
            else:
                _lib.call(entry, *args_before, *args_after)
            torch.cuda.synchronize()
            outs.append(out.clone())
        return outs

    e = m.embed_layer
    hoff, hvoc = e.host_meta()
    args_hm = (hoff, hvoc)
    d = m.d
    xl = torch.empty(B, d, device=gpu)
    prep = m.cross_layer.prepared(d)
    cross_args = ((ids.data_ptr(), kind, ids.stride(0), dense.data_ptr(), 13, 13, e.table.data_ptr(),
                   e.field_offsets.data_ptr(), e.field_vocab.data_ptr()),
                  (F, 16, 3, prep.data_ptr(), xl.data_ptr(), d, B, err.data_ptr(), st), xl)
    prev = _lib.set_option(_lib.OPT_CROSS_KERNEL, 1)  # the staged-tile form: bit-identical
    try:
        a, b = both("rs_embed_cross_fwd", *cross_args)
    finally:
        _lib.set_option(_lib.OPT_CROSS_KERNEL, prev)
    assert torch.equal(a, b) and int(err.item()) == 0
    _lib.set_option(_lib.OPT_CROSS_KERNEL, 0)  # the register form: the same up to G's summation order
    try:
        _, c = both("rs_embed_cross_fwd", *cross_args)
    finally:
        _lib.set_option(_lib.OPT_CROSS_KERNEL, prev)
    assert_scaled_close(c, a.double().cpu().numpy(), rtol=1e-6, what="cross register form vs staged tile")
    assert int(err.item()) == 0
    cross, mlp, dims, acts, _ = m._fused_params()
    n = len(dims) - 1
    y = torch.empty(B, 1, device=gpu)
    dcn_args = ((ids.data_ptr(), kind, ids.stride(0), dense.data_ptr(), 13, 13, e.table.data_ptr(),
                 e.field_offsets.data_ptr(), e.field_vocab.data_ptr()),
                (F, 16, 3, cross.data_ptr(), n, (C.c_int * (n + 1))(*dims), (C.c_int * n)(*acts), mlp.data_ptr(),
                 y.data_ptr(), B, err.data_ptr(), st), y)
    prev = _lib.set_option(_lib.OPT_CROSS_KERNEL, 1)
    try:
        a, b = both("rs_dcn_fwd", *dcn_args)
    finally:
        _lib.set_option(_lib.OPT_CROSS_KERNEL, prev)
    assert torch.equal(a, b) and int(err.item()) == 0
    _lib.set_option(_lib.OPT_CROSS_KERNEL, 0)
    try:
        _, c = both("rs_dcn_fwd", *dcn_args)
    finally:
        _lib.set_option(_lib.OPT_CROSS_KERNEL, prev)
    assert_scaled_close(c, a.double().cpu().numpy(), rtol=1e-6, what="DCN register form vs staged tile")
    assert int(err.item()) == 0
    pe = p.embed_layer
    hoff, hvoc = pe.host_meta()
    args_hm = (hoff, hvoc)
    P = F * (F - 1) // 2
    z = torch.empty(B, F * 16 + P, device=gpu)
    a, b = both("rs_embed_inner_fwd", (ids.data_ptr(), kind, ids.stride(0), pe.table.data_ptr(),
                                       pe.field_offsets.data_ptr(), pe.field_vocab.data_ptr()),
                (F, 16, z.data_ptr(), z.stride(0), B, err.data_ptr(), st), z)
    assert torch.equal(a, b) and int(err.item()) == 0
    z2 = torch.empty(B, F * 16 + 2 * P, device=gpu)
    a, b = both("rs_embed_product_fwd", (ids.data_ptr(), kind, ids.stride(0), pe.table.data_ptr(),
                                         pe.field_offsets.data_ptr(), pe.field_vocab.data_ptr()),
                (F, 16, 1, p.outer_product_layer.prepared().data_ptr(), z2.data_ptr(), z2.stride(0), B,
                 err.data_ptr(), st), z2)
    assert torch.equal(a, b) and int(err.item()) == 0
    bad = ids_np.copy()
    bad[B - 1, F - 1] = vocabs[F - 1]
    bad_t = torch.as_tensor(bad, device=gpu).to(dt)
    for entry, extra in (("rs_embed_cross_fwd_hm", None), ("rs_embed_inner_fwd_hm", None)):
        err.zero_()
        if entry == "rs_embed_cross_fwd_hm":
            _lib.call(entry, bad_t.data_ptr(), kind, bad_t.stride(0), dense.data_ptr(), 13, 13, e.table.data_ptr(),
                      e.field_offsets.data_ptr(), e.field_vocab.data_ptr(), *e.host_meta(), F, 16, 3, prep.data_ptr(),
                      xl.data_ptr(), d, B, err.data_ptr(), st)
        else:
            _lib.call(entry, bad_t.data_ptr(), kind, bad_t.stride(0), pe.table.data_ptr(), pe.field_offsets.data_ptr(),
                      pe.field_vocab.data_ptr(), *pe.host_meta(), F, 16, z.data_ptr(), z.stride(0), B, err.data_ptr(),
                      st)
        torch.cuda.synchronize()
        assert int(err.item()) != 0, entry


# --------------------------- fused DeepFM kernel forms (RS_OPT_DEEPFM_KERNEL)
@pytest.mark.parametrize("variant", [0, 1, 2])
@pytest.mark.parametrize("B,id_dtype,hidden,nd", [(4096, np.int32, [256, 128, 64], 13), (4093, np.int64, [248, 160, 8], 13),
                                                  (33, np.float32, [256, 128], 16), (1, np.int32, [256, 128, 64], 13),
                                                  (300, np.int32, [256, 128, 64], 9)])
def test_deepfm_kernel_forms(gpu, mlp_unroll, variant, B, id_dtype, hidden, nd):
    """rs_deepfm_fwd_hm in its forms — 0: split wave roles (loader waves
    gather the rows and the FM while compute waves run the first layer as the
    fields land; the Criteo shape), 1: one role per wave, 2: every wave
    gathers two fields and computes one layer-0 output tile (deepfm_all, the
    Criteo shape) — == the fp64
    oracle (post-sigmoid 1e-5 relative), the FM logit output too, and an
    out-of-range id raises.  Shapes outside the split form's (nd 9 here) run
    the one-role kernel under both values."""
    from recommender_system_amd import DeepFM, _lib
    from tests.helpers import criteo_columns, dnn_params, tables_of
    rng = np.random.default_rng(B + nd)
    vocabs = rng.integers(2, 5000, size=26)
    m = DeepFM(criteo_columns(vocabs, n_dense=nd, embed_dim=16), 10, 1e-4, 1e-4, hidden, 1, "relu", embed_dim=16,
               seed=9)
    with torch.no_grad():
        for l in m.dnn._layers():
            l.bias.uniform_(-0.1, 0.1)
        m.embed_layer.table.mul_(10.0)  # O(0.5) rows: the tower and the FM both matter
    ids = random_ids(rng, B, vocabs, np.int64)
    ids[0] = vocabs - 1
    dense = rng.random((B, nd)).astype(np.float32)
    ids_t = torch.as_tensor(ids, device=gpu).to({np.int32: torch.int32, np.int64: torch.int64,
                                                 np.float32: torch.float32}[id_dtype])
    prev = _lib.set_option(_lib.OPT_DEEPFM_KERNEL, variant)
    try:
        fm = torch.empty(B, 1, device="cuda")
        y = m.forward_fused((torch.as_tensor(dense, device=gpu), ids_t), fm_logit=fm)
        torch.cuda.synchronize()
        hidden_p, out_p = dnn_params(m.dnn)
        p = {"tables": tables_of(m.embed_layer), "w0": m.fm.w0.cpu().numpy(), "w1": m.fm.w1.cpu().numpy(),
             "v": m.fm.v.cpu().numpy(), "dnn_hidden": hidden_p, "dnn_out": out_p}
        ref, ref_fm, _ = O.deepfm(None, p, nd=nd, inputs=(dense, ids))
        assert_rel_close(y, ref, what=f"DeepFM kernel form {variant}")
        assert_scaled_close(fm, ref_fm, what=f"DeepFM kernel form {variant} fm logit")
        bad = ids_t.clone()
        bad[B - 1, 25] = int(vocabs[25])
        with pytest.raises(IndexError):
            m.forward_fused((torch.as_tensor(dense, device=gpu), bad))
    finally:
        _lib.set_option(_lib.OPT_DEEPFM_KERNEL, prev)


# --------------------------- four MFMA accumulation chains (compile-time)
@pytest.mark.parametrize("B,hidden", [(4096, [256, 128, 64]), (333, [248, 160, 8]), (64, [256, 128])])
def test_mfma_chain_kernels_match_oracle(gpu, B, hidden):
    """The contractions accumulate each output tile in four independent MFMA
    chains summed at the end (an fp32 summation order of their own): the fused
    DeepFM in both kernel forms and the FM logit kernel == the fp64 oracle at
    tower widths that do and do not fill whole k-groups."""
    from recommender_system_amd import DeepFM, _lib
    from tests.helpers import criteo_columns, dnn_params, tables_of
    rng = np.random.default_rng(B + len(hidden))
    vocabs = rng.integers(2, 3000, size=26)
    cols = criteo_columns(vocabs, embed_dim=16)
    dfm = DeepFM(cols, 10, 1e-4, 1e-4, hidden, 1, "relu", embed_dim=16, seed=4)
    with torch.no_grad():
        for l in dfm.dnn._layers():
            l.bias.uniform_(-0.1, 0.1)
        dfm.embed_layer.table.mul_(10.0)
    ids_np = random_ids(rng, B, vocabs, np.int64)
    ids = torch.as_tensor(ids_np, device=gpu).to(torch.int32)
    dense_np = rng.random((B, 13)).astype(np.float32)
    dense = torch.as_tensor(dense_np, device=gpu)
    outs = {}
    lib = _lib.lib()
    prev_k = lib.rs_get_option(_lib.OPT_DEEPFM_KERNEL)
    try:
        for form in (0, 1, 2):
            _lib.set_option(_lib.OPT_DEEPFM_KERNEL, form)
            fm = torch.empty(B, 1, device=gpu)
            outs[("deepfm", form)] = dfm.forward_fused((dense, ids), fm_logit=fm).clone()
            outs[("fm", form)] = fm.clone()
        outs["fm_logit"] = dfm.fm_logit((dense, ids)).clone()
        torch.cuda.synchronize()
    finally:
        _lib.set_option(_lib.OPT_DEEPFM_KERNEL, prev_k)
    hidden_p, out_p = dnn_params(dfm.dnn)
    p = {"tables": tables_of(dfm.embed_layer), "w0": dfm.fm.w0.cpu().numpy(), "w1": dfm.fm.w1.cpu().numpy(),
         "v": dfm.fm.v.cpu().numpy(), "dnn_hidden": hidden_p, "dnn_out": out_p}
    ref, ref_fm, _ = O.deepfm(None, p, nd=13, inputs=(dense_np, ids_np))
    for form in (0, 1, 2):
        assert_rel_close(outs[("deepfm", form)], ref, what=f"deepfm form {form}")
        assert_scaled_close(outs[("fm", form)], ref_fm, what=f"deepfm form {form} fm logit")
    assert_scaled_close(outs["fm_logit"], ref_fm, what="fm logit kernel")


# --------------------------- wide dense blocks in the fused DeepFM
@pytest.mark.parametrize("nd,F,B", [(70, 26, 300), (65, 9, 64), (64, 26, 33)])
def test_deepfm_fused_wide_dense(gpu, nd, F, B):
    """rs_deepfm_fwd_hm with more than 16 dense k-steps (nd > 64) and F <= 32:
    the kernarg-metadata body is built for <= 16 dense k-steps, so such shapes
    must take the streaming-dense body — before the fix the dense columns past
    64 were dropped from the FM logit and left stale in the tower's tile."""
    from recommender_system_amd import DeepFM, _lib
    from tests.helpers import criteo_columns, dnn_params, tables_of
    rng = np.random.default_rng(nd * 31 + F)
    vocabs = rng.integers(2, 3000, size=F)
    m = DeepFM(criteo_columns(vocabs, n_dense=nd, embed_dim=16), 10, 1e-4, 1e-4, [128, 64], 1, "relu",
               embed_dim=16, seed=5)
    with torch.no_grad():
        for l in m.dnn._layers():
            l.bias.uniform_(-0.1, 0.1)
        m.embed_layer.table.mul_(10.0)
    assert m.fused_ok()
    ids = random_ids(rng, B, vocabs, np.int32)
    dense = (rng.random((B, nd)) * 2 - 1).astype(np.float32)
    for form in (0, 1, 2):
        prev = _lib.set_option(_lib.OPT_DEEPFM_KERNEL, form)
        try:
            fm = torch.empty(B, 1, device=gpu)
            y = m.forward_fused((torch.as_tensor(dense, device=gpu), torch.as_tensor(ids, device=gpu)), fm_logit=fm)
            torch.cuda.synchronize()
        finally:
            _lib.set_option(_lib.OPT_DEEPFM_KERNEL, prev)
        hidden_p, out_p = dnn_params(m.dnn)
        p = {"tables": tables_of(m.embed_layer), "w0": m.fm.w0.cpu().numpy(), "w1": m.fm.w1.cpu().numpy(),
             "v": m.fm.v.cpu().numpy(), "dnn_hidden": hidden_p, "dnn_out": out_p}
        ref, ref_fm, _ = O.deepfm(None, p, nd=nd, inputs=(dense, ids))
        assert_rel_close(y, ref, what=f"DeepFM nd={nd} F={F} form {form}")
        assert_scaled_close(fm, ref_fm, what=f"DeepFM nd={nd} F={F} form {form} fm logit")


# ------------------------------------------- tower with a folded input affine
@pytest.mark.gpu
@pytest.mark.parametrize("act", ["relu", "prelu"])
def test_tower_input_affine_equals_bn_then_tower(gpu, act):
    """rs_mlp_affine_fwd (DIN.call's BatchNormalization folded into the tower
    launch) is bit-identical to rs_affine_act followed by rs_mlp_fwd, on a
    strided input view."""
    from recommender_system_amd import DNNLayer
    from recommender_system_amd.layers import BatchNormalization
    torch.manual_seed(3)
    buf = torch.randn(1000, 31, device="cuda")
    x = buf[:, 3:28]  # [1000, 25], row stride 31
    dnn = DNNLayer((256, 128, 64), 1, act, seed=2)
    dnn.build(25)
    with torch.no_grad():
        for L in dnn._layers():
            L.bias.uniform_(-0.1, 0.1)
            if L.alpha is not None:
                L.alpha.uniform_(-0.5, 0.5)
    bn = BatchNormalization()
    bn.build(25)
    with torch.no_grad():
        bn.gamma.uniform_(0.5, 1.5)
        bn.beta.uniform_(-0.1, 0.1)
        bn.moving_mean.uniform_(-0.05, 0.05)
        bn.moving_variance.uniform_(0.5, 2.0)
    xa = bn(x)
    inv, shift = bn.affine()
    assert torch.equal(xa, (x * inv) + shift), "rs_affine_act is x * scale, then + shift"
    ref = dnn.tower(xa.contiguous())
    got = dnn.tower(x, in_affine=(inv, shift))
    torch.cuda.synchronize()
    assert torch.equal(got, ref), float((got - ref).abs().max())


@pytest.mark.parametrize("S,B,last,id_dtype,min_blocks", [
    (1, 4096, 4096, torch.int32, 1),
    (2, 4096, 4093, torch.int32, 2),    # ragged last batch (a partial last tile)
    (8, 4096, 1000, torch.int32, 1),
    (8, 2048, 2048, torch.int64, 2),
    (3, 37, 5, torch.int32, 1),          # batches smaller than a tile
])
def test_embed_fm_stream_bit_identical(gpu, S, B, last, id_dtype, min_blocks):
    """rs_embed_fm_fwd_hm_stream (S consecutive batch requests, one launch):
    every batch's logits == rs_embed_fm_fwd_hm on that batch alone, bit for
    bit, and == the fp64 oracle; rows past the last batch's length untouched;
    an out-of-range id in the last batch sets the flag (IndexError)."""
    from recommender_system_amd import DeepFM
    from tests.helpers import criteo_columns, tables_of
    rng = np.random.default_rng(S * 1000 + B + last)
    vocabs = rng.integers(2, 50000, size=26).tolist()
    m = DeepFM(criteo_columns(vocabs, embed_dim=16), 10, 1e-4, 1e-4, [64, 32], 1, "relu", embed_dim=16, seed=6)
    ids = torch.as_tensor(np.stack([random_ids(rng, B, vocabs) for _ in range(S)]), device=gpu).to(id_dtype)
    dense = torch.as_tensor(rng.random((S, B, 13)).astype(np.float32), device=gpu)
    out = torch.full((S, B, 1), 77.0, device=gpu)
    got = m.fm_logit_stream(dense, ids, last_batch=last, min_blocks=min_blocks, out=out)
    tables = tables_of(m.embed_layer)
    c = lambda t: t.detach().cpu().numpy()
    for s in range(S):
        n = B if s < S - 1 else last
        ref = m.fm_logit((dense[s, :n], ids[s, :n]))
        assert torch.equal(got[s, :n], ref), f"batch {s}"
        x64 = np.concatenate([c(dense[s, :n]).astype(np.float64),
                              O.embed_layer(c(ids[s, :n]), tables, np.float64)], 1)
        assert_scaled_close(got[s, :n, 0], O.fm_layer(x64, c(m.fm.w0), c(m.fm.w1), c(m.fm.v))[:, 0],
                            what=f"stream batch {s}")
    assert bool((got[S - 1, last:] == 77.0).all())
    bad = ids.clone()
    bad[S - 1, last - 1, 25] = vocabs[25]
    with pytest.raises(IndexError):
        m.fm_logit_stream(dense, bad, last_batch=last, min_blocks=min_blocks)
