"""Other interaction ops on the per-field gather:
NFM bi-interaction, AFM (InteractionLayer / AttentionLayer / AFMLayer), FFM.

CPU: known-answer tests that pin the oracle restatements (pair-product sum ==
closed-form bi-interaction; AttentionLayer's size-1 softmax == plain sum; FFM
pair loop == closed form; one-hot FFM == gathered FFM).  GPU: every kernel /
model against the fp64 oracle (tolerance contract in tests/helpers.py).
Parity unpinned by the reference itself (TF absent), as for every layer.
"""
import numpy as np
import pytest

from oracle import ctr_oracle as O
from tests.helpers import assert_rel_close, assert_scaled_close, criteo_columns, random_ids

torch = pytest.importorskip("torch")


# ------------------------------------------------------------ CPU: oracle KATs
def test_bi_interaction_equals_pair_sum():
    rng = np.random.default_rng(1)
    e = rng.normal(size=(6, 9, 5))
    np.testing.assert_allclose(O.interaction_layer(e).sum(1), O.bi_interaction(e), rtol=1e-12, atol=1e-13)
    # pair order: row-major (i<j), like InnerProductLayer
    row, col = O.pair_indices(9)
    np.testing.assert_array_equal(O.interaction_layer(e), e[:, row] * e[:, col])


def test_attention_layer_is_sum_over_rows():
    """softmax over the last axis of a [B,P,1] score tensor is exactly 1."""
    rng = np.random.default_rng(2)
    x = rng.normal(size=(4, 10, 3))
    p = {"att_w_kernel": rng.normal(size=(3, 10)), "att_w_bias": rng.normal(size=10),
         "att_h_kernel": rng.normal(size=(10, 1)) * 50, "att_h_bias": rng.normal(size=1)}
    a = O.attention_layer(x, p)
    np.testing.assert_allclose(a, x.sum(1), rtol=1e-12, atol=1e-12)


def test_ffm_closed_form_and_gather():
    """FFMLayer's pair loop == 0.5(|sum F|^2 - sum |F|^2) on the one-hot
    tensordot, and == the gathered rows nd + offset_c + id_c."""
    rng = np.random.default_rng(3)
    nd, dims, k, B = 3, [5, 2, 7], 4, 11
    fn = nd + sum(dims)
    NF = nd + len(dims)
    w0, w, v = rng.normal(size=1), rng.normal(size=(fn, 1)), rng.normal(size=(fn, NF, k))
    dense = rng.random((B, nd))
    ids = np.stack([rng.integers(0, d, B) for d in dims], 1)
    ref = O.ffm_layer(dense, ids, dims, w0, w, v)
    offs = np.concatenate([[0], np.cumsum(dims)[:-1]])
    rows = nd + offs[None, :] + ids
    Fm = np.einsum("bi,ifk->bfk", dense, v[:nd]) + v[rows].sum(1)
    lin = w0 + dense @ w[:nd] + w[rows, 0].sum(1, keepdims=True)
    inter = 0.5 * ((Fm.sum(1) ** 2).sum(1) - (Fm ** 2).sum((1, 2)))
    np.testing.assert_allclose(ref, lin + inter[:, None], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(O.ffm_layer_gather(dense, ids, dims, w0, w, v), ref, rtol=1e-12, atol=1e-12)
    # tf.one_hot: an out-of-range id contributes a zero row, no error
    bad = ids.copy()
    bad[0, 1] = 99
    np.testing.assert_allclose(O.ffm_layer_gather(dense, bad, dims, w0, w, v), O.ffm_layer(dense, bad, dims, w0, w, v),
                               rtol=1e-12, atol=1e-12)


# ------------------------------------------------------------------- GPU
def _tables(layer):
    return [layer.field_table(i).cpu().numpy() for i in range(layer.n_fields)]


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["att", "avg", "max"])
@pytest.mark.parametrize("k,B,id_dtype", [(8, 300, np.int32), (16, 77, np.int64), (5, 4, np.int32)])
def test_afm(gpu, mode, k, B, id_dtype):
    from recommender_system_amd import AFM
    rng = np.random.default_rng(k + B)
    vocabs = rng.integers(2, 3000, size=26)
    m = AFM(criteo_columns(vocabs, embed_dim=k), mode, seed=4)
    with torch.no_grad():
        # O(1) logits: pooled values and head weights scaled up from the
        # Keras inits (whose logits would all sit at ~0), but short of saturation
        m.afm_layer.output_layer.kernel.mul_(3.0)
        m.afm_layer.output_layer.bias.uniform_(-0.5, 0.5)
        m.afm_layer.embed_layer.table.mul_(5.0 if mode == "att" else 20.0)
    ids = random_ids(rng, B, vocabs, id_dtype)
    dense = rng.random((B, 13)).astype(np.float32)
    y = m((dense, ids))
    pooled, head1 = m.afm_layer.pooled((dense, ids))
    L = m.afm_layer
    p = {"tables": _tables(L.embed_layer), "out_kernel": L.output_layer.kernel.cpu().numpy(),
         "out_bias": L.output_layer.bias.cpu().numpy()}
    if mode == "att":
        a = L.attention_layer
        p.update({"att_w_kernel": a.attention_w.kernel.cpu().numpy(), "att_w_bias": a.attention_w.bias.cpu().numpy(),
                  "att_h_kernel": a.attention_h.kernel.cpu().numpy(), "att_h_bias": a.attention_h.bias.cpu().numpy()})
    ref_y, ref_x = O.afm(None, p, mode, inputs=(dense, ids))
    assert_scaled_close(pooled, ref_x, what=f"AFM {mode} pooled")
    assert_rel_close(y, ref_y, what=f"AFM {mode} output")
    assert_rel_close(head1, O.sigmoid(O.dense(ref_x, p["out_kernel"], p["out_bias"])), what="AFMLayer output")


@pytest.mark.gpu
def test_interaction_and_attention_layers(gpu):
    from recommender_system_amd import AttentionLayer, InteractionLayer
    rng = np.random.default_rng(9)
    e = rng.normal(size=(33, 26, 8)).astype(np.float32)
    pairs = InteractionLayer()(torch.as_tensor(e, device=gpu))
    np.testing.assert_array_equal(pairs.cpu().numpy(), O.interaction_layer(e, np.float32))
    att = AttentionLayer(seed=1)
    out = att(pairs)
    w = att.keras_weights()
    p = {"att_w_kernel": w["dense/kernel"].cpu().numpy(), "att_w_bias": w["dense/bias"].cpu().numpy(),
         "att_h_kernel": w["dense_1/kernel"].cpu().numpy(), "att_h_bias": w["dense_1/bias"].cpu().numpy()}
    assert_scaled_close(out, O.attention_layer(O.interaction_layer(e), p), what="AttentionLayer")


@pytest.mark.gpu
@pytest.mark.parametrize("k,B,id_dtype,hidden", [(8, 500, np.int32, [256, 128, 64]), (16, 33, np.int64, [32]),
                                                 (4, 3, np.int32, [8, 8])])
def test_nfm(gpu, k, B, id_dtype, hidden):
    from recommender_system_amd import NFM
    from tests.helpers import dnn_params
    rng = np.random.default_rng(k * 7 + B)
    vocabs = rng.integers(2, 5000, size=26)
    m = NFM(criteo_columns(vocabs), hidden, 1, embed_dim=k, seed=8)
    with torch.no_grad():
        m.emb_layers.table.mul_(8.0)
        m.bn_layer.moving_mean.uniform_(-0.1, 0.1)
        m.bn_layer.moving_variance.uniform_(0.5, 2.0)
    ids = random_ids(rng, B, vocabs, id_dtype)
    dense = rng.random((B, 13)).astype(np.float32)
    X = np.concatenate([dense, ids.astype(np.float32)], 1)
    y = m(X)
    x_in = m.bi_interaction_input((dense, ids))
    hidden_p, out_p = dnn_params(m.dnn_layers)
    bn = m.bn_layer
    p = {"tables": _tables(m.emb_layers), "bn_mean": bn.moving_mean.cpu().numpy(),
         "bn_var": bn.moving_variance.cpu().numpy(), "bn_gamma": bn.gamma.cpu().numpy(),
         "bn_beta": bn.beta.cpu().numpy(), "dnn_hidden": hidden_p, "dnn_out": out_p,
         "out_kernel": m.output_layer.kernel.cpu().numpy(), "out_bias": m.output_layer.bias.cpu().numpy()}
    ref_y, ref_emb = O.nfm(None, p, inputs=(dense, ids))
    assert_scaled_close(x_in[:, 13:], ref_emb, what="NFM bi-interaction")
    np.testing.assert_array_equal(x_in[:, :13].cpu().numpy(), dense)
    assert_rel_close(y, ref_y, what="NFM output")


@pytest.mark.gpu
@pytest.mark.parametrize("k,B,nvoc,id_dtype", [(8, 200, 300, np.int32), (4, 31, 1000, np.int64),
                                               (16, 7, 50, np.float32), (2, 33, 200, np.int32)])
def test_ffm(gpu, k, B, nvoc, id_dtype):
    from recommender_system_amd import FFM
    rng = np.random.default_rng(k + B)
    vocabs = rng.integers(2, nvoc, size=26)
    m = FFM(criteo_columns(vocabs), k, seed=3)
    ids = random_ids(rng, B, vocabs, np.int64)
    dense = rng.random((B, 13)).astype(np.float32)
    ids_in = ids.astype(id_dtype)
    y = m((dense, ids_in))
    logit = m.ffm((dense, ids_in))
    p = {"w0": m.ffm.w0.cpu().numpy(), "w": m.ffm.w.cpu().numpy(), "v": m.ffm.v.cpu().numpy()}
    ref_logit = O.ffm_layer(dense, ids, list(vocabs), p["w0"], p["w"], p["v"])
    assert_scaled_close(logit, ref_logit, what="FFMLayer logit")
    assert_rel_close(y, O.sigmoid(ref_logit), what="FFM output")
    # the reference's packed X[B,39] and an out-of-range id (tf.one_hot: zero row, no error)
    X = np.concatenate([dense, ids.astype(np.float32)], 1)
    X[0, 13 + 4] = float(vocabs[4] + 3)
    ids_bad = ids.copy()
    ids_bad[0, 4] = vocabs[4] + 3
    assert_rel_close(m(X), O.sigmoid(O.ffm_layer(dense, ids_bad, list(vocabs), p["w0"], p["w"], p["v"])),
                     what="FFM packed X with an out-of-range id")
