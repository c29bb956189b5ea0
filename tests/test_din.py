"""DIN model end to end (a15: model/din.py:15-95) against the oracle's
O.din, which restates DIN.call op for op (Keras Embedding / Attention / BN at
inference / PReLU or Dice Dense / sigmoid).

GPU: the config-4 shape (Amazon-Electronics-shaped: B 2048, T 100, k 8,
behaviour vocab 63,001, 1 dense + a user-id sparse feature of 192,404 ids),
padded histories and a fully padded row, non-trivial BatchNormalization
moving statistics, random PReLU / Dice parameters; dnn_activation 'prelu' and
'dice'; two behaviour features (item + category ids concatenated along k,
model/din.py:73,77-79); attention depths other than the reference's two
hidden layers.  Post-sigmoid outputs at 1e-5 relative."""
import ctypes as ct

import numpy as np
import pytest
import torch

from oracle import ctr_oracle as O
from tests.helpers import assert_rel_close, assert_scaled_close

C = lambda t: t.detach().cpu().numpy()


def din_columns(n_behaviour, k, item_vocab=63001, cate_vocab=801, user_vocab=192404):
    dense = [{"feat": "price"}]
    sparse = [{"feat": "user_id", "feat_onehot_dim": user_vocab, "embed_dim": k},
              {"feat": "movie_seq", "feat_onehot_dim": item_vocab, "embed_dim": k}]
    if n_behaviour > 1:
        sparse.append({"feat": "cate_seq", "feat_onehot_dim": cate_vocab, "embed_dim": k})
    behaviour = [f["feat"] for f in sparse[1:]]
    return [dense, sparse], behaviour


def din_inputs(rng, cols, behaviour, B, T):
    dense, sparse = cols
    lens = rng.integers(1, T + 1, size=B)
    lens[0] = 0  # fully padded history -> uniform average of the padding rows
    lens[1] = T
    valid = np.arange(T)[None, :] < lens[:, None]
    inputs = {}
    for f in sparse:
        V = f["feat_onehot_dim"]
        if f["feat"] in behaviour:
            inputs[f["feat"]] = np.where(valid, rng.integers(1, V, size=(B, T)), 0).astype(np.int64)
        else:
            inputs[f["feat"]] = rng.integers(0, V, size=(B, 1)).astype(np.int64)
    for f in dense:
        inputs[f["feat"]] = rng.random((B, 1)).astype(np.float32)
    vocab = {f["feat"]: f["feat_onehot_dim"] for f in sparse}
    cand = np.stack([rng.integers(0, vocab[b], size=B) for b in behaviour], 1)
    cand[2] = [vocab[b] - 1 for b in behaviour]  # last row of each behaviour table
    inputs["movie_id"] = cand.astype(np.int64)
    return inputs


def randomize(model, rng):
    """Non-trivial values for every parameter the reference initialises to a
    constant (PReLU / Dice alphas, BN statistics, biases)."""
    u = lambda t, lo, hi: t.copy_(torch.as_tensor(rng.uniform(lo, hi, size=tuple(t.shape)), dtype=torch.float32))
    with torch.no_grad():
        for L in model.embed_seq_layers:
            L.table.mul_(10.0)  # O(0.5) embeddings: the attention scores spread
        att = model.att_layer
        for a in att.alphas:
            u(a, -0.5, 0.5)
        for b in att.biases:
            u(b, -0.1, 0.1)
        for d in att.dice:
            u(d.alphas, -0.5, 0.5)
            u(d.moving_mean, -0.1, 0.1)
            u(d.moving_variance, 0.5, 1.5)
        bn = model.bn_layer
        u(bn.gamma, 0.5, 1.5)
        u(bn.beta, -0.1, 0.1)
        u(bn.moving_mean, -0.05, 0.05)
        u(bn.moving_variance, 0.5, 2.0)
        for L in list(model.dense_layer) + [model.out_layer]:
            u(L.bias, -0.1, 0.1)
            if L.alpha is not None:
                u(L.alpha, -0.5, 0.5)
            if L.dice is not None:
                u(L.dice.alphas, -0.5, 0.5)
                u(L.dice.moving_mean, -0.2, 0.2)
                u(L.dice.moving_variance, 0.5, 1.5)
    model._weights_changed()


def din_params(model):
    att = model.att_layer
    p_att = {"out": (C(att.out_kernel), C(att.out_bias))}
    if att.activation == "prelu":
        p_att["prelu"] = [(C(att.kernels[i]), C(att.biases[i]), C(att.alphas[i])) for i in range(len(att.kernels))]
    else:
        p_att["dice"] = [(C(d.alphas), C(d.moving_mean), C(d.moving_variance), d.epsilon) for d in att.dice]
    dnn = []
    for L in model.dense_layer:
        ap = C(L.alpha) if L.activation == "prelu" else (C(L.dice.alphas), C(L.dice.moving_mean),
                                                          C(L.dice.moving_variance), L.dice.epsilon)
        dnn.append((C(L.kernel), C(L.bias), ap))
    bn = model.bn_layer
    return {"sparse_tables": {f["feat"]: L.field_table(0).cpu().numpy()
                              for f, L in zip(model.other_sparse, model.embed_sparse_layers)},
            "seq_tables": {f["feat"]: L.field_table(0).cpu().numpy()
                           for f, L in zip(model.seq_feats, model.embed_seq_layers)},
            "att": p_att, "bn": (C(bn.gamma), C(bn.beta), C(bn.moving_mean), C(bn.moving_variance), bn.epsilon),
            "dnn": dnn, "out": (C(model.out_layer.kernel), C(model.out_layer.bias))}


@pytest.mark.gpu
@pytest.mark.parametrize("dnn_act,att_act,att_hidden,nb,k,B,T", [
    ("prelu", "prelu", (80, 40), 1, 8, 2048, 100),     # config 4, the reference's defaults (id-driven attention)
    ("dice", "prelu", (80, 40), 1, 8, 2048, 100),      # config 4, dnn_activation='dice'
    ("prelu", "prelu", (80, 40), 2, 8, 512, 100),      # item + category behaviour (K = 16, fused attention)
    ("dice", "dice", (80, 40), 2, 8, 300, 30),         # att_attention='dice' on two behaviour features
    ("prelu", "prelu", (64,), 1, 8, 256, 100),         # one attention hidden layer (generic path)
    ("prelu", "prelu", (80, 40, 20), 2, 4, 256, 50),   # three hidden layers (generic path), K = 8
    ("prelu", "prelu", (200, 40), 1, 8, 128, 20),      # H > 128 (generic path)
])
def test_din_model(gpu, dnn_act, att_act, att_hidden, nb, k, B, T):
    from recommender_system_amd import DIN
    rng = np.random.default_rng(B + T + nb * 7 + len(att_hidden))
    cols, behaviour = din_columns(nb, k)
    model = DIN(cols, behaviour, att_hidden_units=att_hidden, att_attention=att_act, dnn_activation=dnn_act,
                seed=11)
    inputs = din_inputs(rng, cols, behaviour, B, T)
    model(inputs)  # builds the lazily-shaped layers (Keras build on first call)
    randomize(model, rng)
    y = model(inputs)
    sparse = [f["feat"] for f in cols[1]]
    ref, att = O.din(inputs, din_params(model), [f["feat"] for f in cols[0]], sparse,
                     [f for f in sparse if f in behaviour], att_act=att_act, dnn_act=dnn_act)
    assert_rel_close(y, ref, what=f"DIN {dnn_act}/{att_act} {att_hidden} nb={nb}")
    # the fully padded row attends uniformly; its output is still finite
    assert np.isfinite(y.cpu().numpy()).all()


@pytest.mark.gpu
@pytest.mark.parametrize("nb", [1, 2])
def test_din_model_bad_ids(gpu, nb):
    """An out-of-range behaviour / candidate id raises IndexError (Keras
    Embedding's InvalidArgumentError on CPU) — nb = 1 is the id-driven path
    whose one launch also copies the candidate rows."""
    from recommender_system_amd import DIN
    rng = np.random.default_rng(5)
    cols, behaviour = din_columns(nb, 8)
    model = DIN(cols, behaviour, seed=1)
    inputs = din_inputs(rng, cols, behaviour, 64, 20)
    model(inputs)
    for key, val in ((behaviour[-1], 801 if nb == 2 else 63001), ("movie_id", 63001), ("user_id", 192404)):
        bad = {k_: v.copy() for k_, v in inputs.items()}
        if key == "movie_id":
            bad[key][3, 0] = val
        else:
            bad[key][3, 0] = val
        with pytest.raises(IndexError):
            model(bad)


@pytest.mark.gpu
@pytest.mark.parametrize("nb,B,T", [(1, 2048, 100), (2, 37, 20)])
def test_din_tower_reads_pieces(gpu, nb, B, T):
    """DIN.call's tower reading the other sparse embeddings and the dense
    features itself (rs_mlp_affine_pieces_fwd: no rs_concat_pieces launch, no
    concat buffer) == the two-launch form (concat, then the tower), bit for
    bit — the staged values and the arithmetic are the same."""
    from recommender_system_amd import DIN
    rng = np.random.default_rng(B + nb)
    cols, behaviour = din_columns(nb, 8)
    model = DIN(cols, behaviour, seed=3)
    inputs = din_inputs(rng, cols, behaviour, B, T)
    model(inputs)
    randomize(model, rng)
    y1 = model(inputs)
    model.pieces_in_tower = False
    y0 = model(inputs)
    assert torch.equal(y1, y0)


@pytest.mark.gpu
@pytest.mark.parametrize("k,B,T,idt", [(8, 2048, 100, np.int64), (8, 1003, 100, np.int32), (4, 37, 20, np.int64),
                                       (16, 203, 128, np.int32), (8, 5, 7, np.float32)])
def test_din_one_launch_matches_two(gpu, k, B, T, idt):
    """DIN.call as ONE launch (rs_din_forward_ids: the attention unit, then bn
    + the PReLU tower + Dense(1, sigmoid) in the same workgroups, 8 samples
    each on a 16-row tile) == the attention launch + the tower launch, bit for
    bit: ragged batches, k 4 / 8 / 16, 1..8 position tiles, int32 / int64 /
    float ids; and an out-of-range id of a piece (the user_id embedding read
    inside the tower staging) raises."""
    from recommender_system_amd import DIN, _lib
    rng = np.random.default_rng(B + k)
    cols, behaviour = din_columns(1, k)
    model = DIN(cols, behaviour, seed=5)
    inputs = din_inputs(rng, cols, behaviour, B, T)
    model(inputs)
    randomize(model, rng)
    inputs = {f: (v.astype(idt) if f != "price" else v) for f, v in inputs.items()}
    dims = model._dims()
    assert _lib.lib().rs_din_forward_ids_supported(T, k, 80, 40, len(dims) - 1, (ct.c_int * len(dims))(*dims)) == 1
    y1 = model(inputs)
    model.fused_call = False
    y0 = model(inputs)
    assert torch.equal(y1, y0)
    model.fused_call = True
    bad = dict(inputs)
    bad["user_id"] = inputs["user_id"].copy()
    bad["user_id"][B // 2] = 192404
    with pytest.raises(IndexError):
        model(bad)
    assert torch.equal(model(inputs), y1)  # the flag was cleared by the raise


def test_oracle_din_two_behaviours_is_concat():
    """CPU: O.din with two behaviour features equals the attention over the
    k-concatenated embeddings with the mask of the first feature."""
    rng = np.random.default_rng(3)
    B, T, k = 6, 7, 4
    cols, behaviour = din_columns(2, k, item_vocab=50, cate_vocab=9, user_vocab=11)
    inputs = din_inputs(rng, cols, behaviour, B, T)
    tabs = {f["feat"]: rng.standard_normal((f["feat_onehot_dim"], k)) for f in cols[1]}
    att = {"prelu": [(rng.standard_normal((8 * k, 5)), rng.standard_normal(5), rng.standard_normal((T, 5)))],
           "out": (rng.standard_normal((5, 1)), rng.standard_normal(1))}
    width = 2 * 2 * k + k + 1
    p = {"sparse_tables": {"user_id": tabs["user_id"]}, "seq_tables": {b: tabs[b] for b in behaviour}, "att": att,
         "bn": (np.ones(width), np.zeros(width), np.zeros(width), np.ones(width), 1e-3),
         "dnn": [(rng.standard_normal((width, 3)), np.zeros(3), np.zeros(3))],
         "out": (rng.standard_normal((3, 1)), np.zeros(1))}
    _, a = O.din(inputs, p, ["price"], ["user_id"] + behaviour, behaviour)
    seq = np.concatenate([tabs[b][inputs[b]] for b in behaviour], -1)
    item = np.concatenate([tabs[b][inputs["movie_id"][:, i]] for i, b in enumerate(behaviour)], -1)
    mask = (inputs[behaviour[0]] != 0).astype(np.float64)
    np.testing.assert_allclose(a, O.attention(item, seq, seq, mask, att), rtol=1e-12)
    np.testing.assert_allclose(a[0], seq[0].mean(0), rtol=1e-12)  # fully padded row: uniform average


def _cp(x):
    if isinstance(x, np.ndarray):
        return x.copy()
    if isinstance(x, tuple):
        return tuple(_cp(y) for y in x)
    return x


def _din_train_params(model):
    p = din_params(model)
    att = {k_: [_cp(l) for l in v] for k_, v in p["att"].items() if k_ != "out"}
    att["out"] = _cp(p["att"]["out"])
    return {"sparse_tables": {f: v.copy() for f, v in p["sparse_tables"].items()},
            "seq_tables": {f: v.copy() for f, v in p["seq_tables"].items()},
            "att": att, "bn": _cp(p["bn"]), "dnn": [_cp(l) for l in p["dnn"]], "out": _cp(p["out"])}


def _flat_params(p):
    out = {f"sparse/{f}": v for f, v in p["sparse_tables"].items()}
    out.update({f"seq/{f}": v for f, v in p["seq_tables"].items()})
    for i, l in enumerate(p["att"].get("prelu", [])):
        out.update({f"att{i}/W": l[0], f"att{i}/b": l[1], f"att{i}/alpha": l[2]})
    for i, l in enumerate(p["att"].get("dice", [])):
        out.update({f"att_dice{i}/alpha": l[0], f"att_dice{i}/mean": l[1], f"att_dice{i}/var": l[2]})
    out.update({"att_out/W": p["att"]["out"][0], "att_out/b": p["att"]["out"][1]})
    out.update({f"bn/{n}": v for n, v in zip(("gamma", "beta", "mean", "var"), p["bn"][:4])})
    for i, l in enumerate(p["dnn"]):
        out.update({f"dnn{i}/W": l[0], f"dnn{i}/b": l[1]})
        if isinstance(l[2], tuple):  # Dice: alpha, moving mean, moving var
            out.update({f"dnn{i}/alpha": l[2][0], f"dnn{i}/mean": l[2][1], f"dnn{i}/var": l[2][2]})
        else:
            out[f"dnn{i}/alpha"] = l[2]
    out.update({"out/W": p["out"][0], "out/b": p["out"][1]})
    return out


def _assert_update_close(got, ref, before, rtol=2e-3, what=""):
    """(got - before) vs (ref - before) at rtol of the update's scale, plus
    the fp32 storage quantum of the parameter (4 ulp of |before|): an update
    far below a parameter's ulp is only as exact as fp32 can hold it.  1e-8
    absolute floor: the attention's output bias has an exactly-zero gradient
    (softmax is shift invariant), 1e-19 in the fp64 oracle."""
    got, ref, before = (np.asarray(v, np.float64) for v in (got, ref, before))
    dg, dr = got - before, ref - before
    rms = float(np.sqrt(np.mean(dr ** 2)))
    bound = rtol * np.maximum(np.abs(dr), rms) + 4 * np.finfo(np.float32).eps * np.abs(before) + 1e-8
    bad = ~(np.abs(dg - dr) <= bound)
    assert not bad.any(), f"{what}: {int(bad.sum())}/{bad.size} outside tolerance"


@pytest.mark.gpu
@pytest.mark.parametrize("att_hidden,dnn_hidden,nb,k,B,T,att_act,dnn_act,fused,rate", [
    ((80, 40), (256, 128, 64), 1, 8, 256, 20, "prelu", "prelu", True, 0.0),   # the reference defaults
    ((80, 40), (256, 128, 64), 1, 8, 256, 20, "prelu", "prelu", True, 0.2),   # ... with dnn_dropout=0.2
    ((80, 40), (64, 32), 1, 8, 256, 20, "prelu", "dice", True, 0.2),          # dropout after a Dice DNN
    ((80, 40), (256, 128, 64), 1, 8, 256, 20, "prelu", "prelu", False, 0.0),  # ... attention unit layer by layer
    ((80, 40), (64, 32), 2, 8, 192, 30, "prelu", "prelu", True, 0.0),         # item + category features (K = 16)
    ((80, 40), (64, 32), 1, 8, 40, 100, "prelu", "prelu", True, 0.0),         # config 4's T = 100 (Rp = 112)
    ((56, 24), (16,), 1, 8, 30, 128, "prelu", "prelu", True, 0.0),            # T = 128, widths with pads
    ((80, 40), (64, 32), 1, 8, 300, 7, "prelu", "prelu", True, 0.0),          # T = 7: one row tile, > 256 samples
    ((32,), (16,), 2, 4, 64, 7, "prelu", "prelu", True, 0.0),                 # one attention layer, small ragged T
    ((80, 40), (64, 32), 1, 8, 256, 20, "prelu", "dice", True, 0.0),          # dnn_activation='dice'
    ((80, 40), (64, 32), 2, 8, 128, 30, "dice", "dice", True, 0.0),           # att_attention='dice' too
])
def test_din_train_steps_match_oracle(gpu, att_hidden, dnn_hidden, nb, k, B, T, att_act, dnn_act, fused, rate):
    """DIN.train_step (compile_fit on DIN in training mode: batch-statistics
    BatchNormalization with moving averages, PReLU attention over [T, h]
    alphas, masked softmax pool, PReLU DNN, SGD + row-sparse embedding SGD)
    == oracle.din_train_step (pinned by finite differences) over 3 steps with
    small vocabularies (repeated rows, candidates inside the histories), a
    fully padded history row and non-trivial parameters.  Parameters and the
    per-step updates are compared at 2e-3 of their scale.  ``fused``: the
    two-layer PReLU attention's backward as one rs_din_att_prelu_bwd launch
    and its forward as one rs_din_att_prelu_fwd launch (False: layer by layer).
    ``rate``: DIN(dnn_dropout=rate) — the Dropout after the DNN (din.py:93)
    in training mode, the oracle fed the same multiplier."""
    from recommender_system_amd import DIN
    from recommender_system_amd import models as M
    from tests.helpers import dropout_masks
    rng = np.random.default_rng(B + T + nb)
    cols, behaviour = din_columns(nb, k, item_vocab=40, cate_vocab=9, user_vocab=17)
    model = DIN(cols, behaviour, att_hidden_units=att_hidden, dnn_hidden_units=dnn_hidden, att_attention=att_act,
                dnn_activation=dnn_act, dnn_dropout=rate, seed=3)
    model.fused_att_train = fused
    if fused and att_act == "prelu" and len(att_hidden) == 2:  # the shape takes the fused kernel
        from recommender_system_amd import _lib
        assert _lib.lib().rs_din_att_prelu_bwd_workspace_size(B, T, 4 * k * nb, *att_hidden) > 0
    inputs = din_inputs(rng, cols, behaviour, B, T)
    model(inputs)
    randomize(model, rng)
    dense_f = [f["feat"] for f in cols[0]]
    sparse_f = [f["feat"] for f in cols[1]]
    beh = [f for f in sparse_f if f in behaviour]
    p = _din_train_params(model)
    lr = 0.2
    for step in range(3):
        inputs = din_inputs(rng, cols, behaviour, B, T)
        t = rng.integers(0, 2, B).astype(np.float32)
        before = _flat_params(_din_train_params(model))
        drop_mask = None
        if rate:
            dr = M._dropout_rng(model)
            drop_mask = dropout_masks(dr.seed, dr.offset, B, [dnn_hidden[-1]], rate)[0][0]
        loss = model.train_step(inputs, t, lr=lr, return_loss=True)
        p, ce = O.din_train_step(inputs, t, p, dense_f, sparse_f, beh, lr, att_act=att_act, dnn_act=dnn_act,
                                 drop_mask=drop_mask)
        got = _flat_params(_din_train_params(model))
        ref = _flat_params(p)
        assert_scaled_close(loss, ce, rtol=1e-4, what=f"step {step} loss")
        for name in ref:
            _assert_update_close(got[name], ref[name], before[name], what=f"step {step} update {name}")
        p = _din_train_params(model)  # next step from the same fp32 point
    # the inference forward on the trained weights (packed attention images
    # rebuilt after the raw-pointer updates; BN on the moved averages)
    ref, _ = O.din(inputs, din_params(model), dense_f, sparse_f, beh, att_act=att_act, dnn_act=dnn_act)
    assert_rel_close(model(inputs), ref, what="forward after training")
