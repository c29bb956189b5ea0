"""CPU oracle for the CTR forward path — TEST INFRASTRUCTURE ONLY.

This module is a numpy op-for-op restatement of the reference's TF2/Keras
forward path (Hcyand/recommender_system, algorithm/deep_learning/...).  Only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import it, and only as the checker / the timed CPU baseline.  The product
path (``recommender_system_amd``) never imports it and has no CPU fallback.

PARITY STATUS: the reference's layer/model arithmetic lives in TensorFlow/Keras
(unpinned TF 2.x), which is not installed in this image (ImportError, no
network).  The layer math below is therefore **parity unpinned** by the
reference itself: it is pinned by known-answer tests (brute-force FM pairwise
sum, explicit per-sample CrossNet loop, per-pair inner products, one-hot FM ==
gather FM, attention with one / zero unmasked positions; see
tests/test_oracle.py).  The input producer (utils/dataset.py) IS pinned against
the reference itself: tests/golden/make_golden.py imports the reference's
``utils/dataset.py`` in the build container and commits its outputs as
fixtures.

Keras semantics restated here (third-party behaviour the reference relies on):
  * Model inputs are autocast to float32 (``cast_inputs``).
  * ``Embedding`` casts float ids to int32 by truncation, raises on an id outside
    [0, vocab) (TF CPU InvalidArgumentError -> IndexError here).
  * ``Dense`` kernel is (in, out); a 3-D input is a tensordot over its last axis.
  * ``PReLU()`` alpha has shape input_shape[1:] (shared_axes=None).
  * ``BatchNormalization`` at inference: (x - moving_mean)/sqrt(moving_var+eps)
    * gamma + beta (eps 1e-3 default; Dice uses eps 1e-9, center/scale off).
  * ``Dropout`` is the identity at inference.
  * ``-2**32 + 1`` is -4294967295, which rounds to -4294967296.0 in float32.

All functions take a ``dt`` argument (np.float64 for golden vectors, np.float32
for the timed CPU baseline) and compute in that dtype.
"""
from __future__ import annotations

import numpy as np

MASK_FILL = -2 ** 32 + 1  # layer/interaction.py:399


# ----------------------------------------------------------------- helpers
def cast_inputs(x, dt=np.float32):
    """Keras Model.__call__ autocast of floating inputs (float64 -> float32)."""
    return np.asarray(x, dtype=np.float32).astype(dt)


def cast_ids(ids):
    """Keras Embedding: ``tf.cast(inputs, 'int32')`` for non-integer ids
    (truncation toward zero); integer ids pass through unchanged."""
    ids = np.asarray(ids)
    if np.issubdtype(ids.dtype, np.floating):
        with np.errstate(invalid="ignore"):
            return np.trunc(ids.astype(np.float32)).astype(np.int64)
    return ids.astype(np.int64)


def embedding_lookup(table, ids):
    """tf.gather(table, ids) with TF-CPU's out-of-range error."""
    ids = cast_ids(ids)
    if ids.size and (ids.min() < 0 or ids.max() >= table.shape[0]):
        raise IndexError(f"embedding id out of range [0, {table.shape[0]})")
    return table[ids]


# ----------------------------------------------------- layers (a3 .. a14)
def embed_layer(sparse, tables, dt=np.float64):
    """EmbedLayer.call (layer/core.py:273-280): per-field Embedding, stack to
    [F,B,k], transpose to [B,F,k], reshape to [B,F*k] (field-major)."""
    sparse = np.asarray(sparse)
    embs = [embedding_lookup(np.asarray(t, dt), sparse[:, i]) for i, t in enumerate(tables)]
    emb = np.transpose(np.stack(embs, 0), (1, 0, 2))
    return emb.reshape(emb.shape[0], emb.shape[1] * emb.shape[2])


def fm_layer(x, w0, w1, v, dt=np.float64):
    """FMLayer.call (layer/interaction.py:106-114), op for op."""
    x = np.asarray(x, dt)
    w0, w1, v = (np.asarray(a, dt) for a in (w0, w1, v))
    linear = x @ w1.reshape(-1, 1) + w0.reshape(1)
    p1 = np.power(x @ v, 2)
    p2 = np.power(x, 2) @ np.power(v, 2)
    inter = 0.5 * np.sum(p1 - p2, axis=-1, keepdims=True)
    return linear + inter


def fm_layer_pairwise(x, w0, w1, v, dt=np.float64):
    """Known-answer form of the FM: w0 + x.w1 + sum_{i<j} <v_i,v_j> x_i x_j."""
    x = np.asarray(x, dt)
    v = np.asarray(v, dt)
    gram = v @ v.T
    iu = np.triu_indices(v.shape[0], 1)
    w0 = np.asarray(w0, dt).reshape(-1)[0]
    w1 = np.asarray(w1, dt).reshape(-1)
    out = np.empty((x.shape[0], 1), dt)
    for b in range(x.shape[0]):
        xx = np.outer(x[b], x[b])
        out[b, 0] = w0 + x[b] @ w1 + np.sum(gram[iu] * xx[iu])
    return out


def fm_onehot_gather(dense, ids, field_offsets, w0, w1, v, dt=np.float64):
    """FM model on one-hot x, computed as a gather (model/fm.py + the identity
    x[b, nd + off_c + id_c] = 1, utils/dataset.py:47-48)."""
    dense = np.asarray(dense, dt)
    ids = cast_ids(ids)
    nd = dense.shape[1]
    rows = nd + np.asarray(field_offsets)[None, :] + ids
    v = np.asarray(v, dt)
    w1 = np.asarray(w1, dt).reshape(-1)
    s = dense @ v[:nd] + v[rows].sum(1)
    q = (dense ** 2) @ (v[:nd] ** 2) + (v[rows] ** 2).sum(1)
    lin = dense @ w1[:nd] + w1[rows].sum(1) + np.asarray(w0, dt).reshape(1)
    return (lin + 0.5 * np.sum(s * s - q, axis=1)).reshape(-1, 1)


def activation(x, act, alpha=None):
    if act is None or act == "linear":
        return x
    if act == "relu":
        return np.maximum(x, 0)
    if act == "sigmoid":
        return 1.0 / (1.0 + np.exp(-x))
    if act == "prelu":
        return prelu(x, alpha)
    raise ValueError(act)


def prelu(x, alpha):
    """Keras PReLU: max(0,x) + alpha * min(0,x) (alpha broadcast from the
    trailing dims, shape input_shape[1:])."""
    return np.maximum(x, 0) + alpha * np.minimum(x, 0)


def dense(x, kernel, bias, act=None, alpha=None, dt=np.float64):
    """Keras Dense: tensordot(x, kernel, [[-1],[0]]) + bias, then activation."""
    x = np.asarray(x, dt)
    y = np.tensordot(x, np.asarray(kernel, dt), axes=[[x.ndim - 1], [0]]) + np.asarray(bias, dt)
    return activation(y, act, None if alpha is None else np.asarray(alpha, dt))


def dnn_layer(x, hidden, out, act="relu", dt=np.float64):
    """DNNLayer.call (layer/interaction.py:40-46); Dropout is inactive."""
    for kern, bias in hidden:
        x = dense(x, kern, bias, act, dt=dt)
    return dense(x, out[0], out[1], None, dt=dt)


def cross_layer(x, ws, bs, dt=np.float64):
    """CrossLayer.call (layer/interaction.py:75-83), op for op on [B,d,1]."""
    x0 = np.asarray(x, dt)[:, :, None]
    x1 = x0
    for w, b in zip(ws, bs):
        w = np.asarray(w, dt).reshape(-1, 1)
        b = np.asarray(b, dt).reshape(-1, 1)
        x1_w = np.matmul(np.transpose(x1, (0, 2, 1)), w)  # [B,1,1]
        x1 = np.matmul(x0, x1_w) + b + x1
    return x1[:, :, 0]


def cross_layer_loop(x, ws, bs, dt=np.float64):
    """Known-answer form: explicit per-sample loop of x_{l+1}=x0 (x_l.w)+b+x_l."""
    x = np.asarray(x, dt)
    out = np.empty_like(x)
    for n in range(x.shape[0]):
        x0 = x[n]
        xl = x0.copy()
        for w, b in zip(ws, bs):
            xl = x0 * float(xl @ np.asarray(w, dt).reshape(-1)) + np.asarray(b, dt).reshape(-1) + xl
        out[n] = xl
    return out


def pair_indices(F):
    """Row-major (i<j) pair order of InnerProductLayer (layer/interaction.py:172-177)."""
    row, col = [], []
    for i in range(F - 1):
        for j in range(i + 1, F):
            row.append(i)
            col.append(j)
    return np.array(row), np.array(col)


def inner_product_layer(e, dt=np.float64):
    """InnerProductLayer.call (layer/interaction.py:170-183) on [B,F,k]."""
    e = np.asarray(e, dt)
    row, col = pair_indices(e.shape[1])
    p = e[:, row, :]
    q = e[:, col, :]
    return np.sum(p * q, axis=-1)


def inner_product_loop(e, dt=np.float64):
    e = np.asarray(e, dt)
    B, F, _ = e.shape
    out = []
    for i in range(F - 1):
        for j in range(i + 1, F):
            out.append([float(e[b, i] @ e[b, j]) for b in range(B)])
    return np.asarray(out, dt).T.reshape(B, -1)


def batchnorm_inference(x, mean, var, gamma=None, beta=None, eps=1e-3, dt=np.float64):
    x = np.asarray(x, dt)
    y = (x - np.asarray(mean, dt)) / np.sqrt(np.asarray(var, dt) + dt(eps))
    if gamma is not None:
        y = y * np.asarray(gamma, dt)
    if beta is not None:
        y = y + np.asarray(beta, dt)
    return y


def dice(x, alpha, mean, var, eps=1e-9, dt=np.float64):
    """Dice.call at inference (layer/interaction.py:421-425)."""
    x = np.asarray(x, dt)
    xn = batchnorm_inference(x, mean, var, eps=eps, dt=dt)
    xp = 1.0 / (1.0 + np.exp(-xn))
    return np.asarray(alpha, dt) * (1.0 - xp) * x + xp * x


def attention(query, key, value, mask, params, act="prelu", dt=np.float64):
    """Attention.call (layer/interaction.py:369-406).

    params['prelu'] = [(kernel, bias, alpha[T,h]), ...] ; params['dice'] =
    [(alpha[4k], mean[4k], var[4k], eps), ...] ; params['out'] = (kernel, bias).
    """
    q = np.asarray(query, dt)[:, None, :]
    key = np.asarray(key, dt)
    value = np.asarray(value, dt)
    q = np.tile(q, (1, key.shape[1], 1))
    emb = np.concatenate([q, key, q - key, q * key], axis=-1)
    if act == "prelu":
        for kern, bias, alpha in params["prelu"]:
            emb = dense(emb, kern, bias, "prelu", alpha, dt=dt)
    elif act == "dice":
        for alpha, mean, var, eps in params["dice"]:
            emb = dice(emb, alpha, mean, var, eps, dt=dt)
    else:
        raise ValueError(act)
    score = dense(emb, params["out"][0], params["out"][1], None, dt=dt)[..., 0]
    padding = np.ones_like(score) * dt(np.float32(MASK_FILL))
    score = np.where(np.asarray(mask) == 0, padding, score)
    score = score - score.max(-1, keepdims=True)
    e = np.exp(score)
    score = e / e.sum(-1, keepdims=True)
    return np.matmul(score[:, None, :], value)[:, 0, :]


def sigmoid(x):
    return 1.0 / (1.0 + np.exp(-x))


# ------------------------------------------------------------- models
def fm_model(x, p, dt=np.float64):
    """FM.call (model/fm.py:19-23): sigmoid(FMLayer(x))."""
    return sigmoid(fm_layer(cast_inputs(x, dt), p["w0"], p["w1"], p["v"], dt=dt))


def _split_dense_sparse(X, nd, dt):
    Xc = cast_inputs(X, dt)
    Xf = np.asarray(X, np.float32)  # ids go through the float32 autocast
    return Xc[:, :nd], Xf[:, nd:]


def deepfm(X, p, nd=13, dt=np.float64, inputs=None):
    """DeepFM.call (model/deepFM.py:23-31).  X: packed [B, nd+F] or
    inputs=(dense, ids)."""
    dense_in, sparse = inputs if inputs is not None else _split_dense_sparse(X, nd, dt)
    x = np.concatenate([np.asarray(dense_in, dt), embed_layer(sparse, p["tables"], dt)], axis=-1)
    fm = fm_layer(x, p["w0"], p["w1"], p["v"], dt=dt)
    dnn = dnn_layer(x, p["dnn_hidden"], p["dnn_out"], p.get("act", "relu"), dt=dt)
    return sigmoid(0.5 * (fm + dnn)), fm, x


def dcn(X, p, nd=13, dt=np.float64, inputs=None):
    """DCN.call (model/dcn.py:24-34)."""
    dense_in, sparse = inputs if inputs is not None else _split_dense_sparse(X, nd, dt)
    x = np.concatenate([np.asarray(dense_in, dt), embed_layer(sparse, p["tables"], dt)], axis=1)
    cross = cross_layer(x, p["cross_w"], p["cross_b"], dt=dt)
    dnn = dnn_layer(x, p["dnn_hidden"], p["dnn_out"], p.get("act", "relu"), dt=dt)
    z = np.concatenate([cross, dnn], axis=1)
    return sigmoid(dense(z, p["out_kernel"], p["out_bias"], dt=dt)), cross


def outer_product_layer(e, W, dt=np.float64):
    """OuterProductLayer.call (layer/interaction.py:200-215) op for op:
    p [B,1,P,k] * W [k,P,k] -> sum over the last axis -> [B,k,P] ->
    transpose * q -> sum: out[b,p] = sum_a q[b,p,a] sum_j p[b,p,j] W[a,p,j]."""
    e = np.asarray(e, dt)
    W = np.asarray(W, dt)
    row, col = pair_indices(e.shape[1])
    pp = e[:, row, :][:, None, :, :]           # [B,1,P,k]
    qq = e[:, col, :]                          # [B,P,k]
    tmp = np.sum(pp * W[None], axis=-1)        # [B,k,P]
    return np.sum(np.transpose(tmp, (0, 2, 1)) * qq, axis=-1)


def outer_product_loop(e, W, dt=np.float64):
    """Known-answer restatement: out[b,p] = e_row^T W_p^T e_col per pair."""
    e = np.asarray(e, dt)
    W = np.asarray(W, dt)
    B, F, _ = e.shape
    out = []
    p = 0
    for i in range(F - 1):
        for j in range(i + 1, F):
            Wp = W[:, p, :]                    # [a, j']
            out.append([float(e[b, j] @ (Wp @ e[b, i])) for b in range(B)])
            p += 1
    return np.asarray(out, dt).T.reshape(B, -1)


def pnn(X, p, mode="inner", nd=13, dt=np.float64, inputs=None):
    """PNN.call (model/pnn.py:28-53), mode 'inner' / 'outer' / 'both', with
    3-D embeddings.  p['outer_W'] is the OuterProductLayer weight [k,P,k]."""
    _, sparse = inputs if inputs is not None else _split_dense_sparse(X, nd, dt)
    flat = embed_layer(sparse, p["tables"], dt)
    k = np.asarray(p["tables"][0]).shape[1]
    z = flat.reshape(flat.shape[0], -1, k)
    parts = [flat]
    if mode in ("inner", "both"):
        parts.append(inner_product_layer(z, dt=dt))
    if mode in ("outer", "both"):
        parts.append(outer_product_layer(z, p["outer_W"], dt=dt))
    x = np.concatenate(parts, axis=1)
    return dnn_layer(x, p["dnn_hidden"], p["dnn_out"], p.get("act", "relu"), dt=dt), x


def pnn_inner(X, p, nd=13, dt=np.float64, inputs=None):
    """PNN.call mode='inner' (model/pnn.py:28-53) with 3-D embeddings [B,F,k]
    (documented deviation: the reference's rank-2 EmbedLayer crashes at
    model/pnn.py:38).  Returns the DNN logit (no sigmoid, as the reference)."""
    _, sparse = inputs if inputs is not None else _split_dense_sparse(X, nd, dt)
    flat = embed_layer(sparse, p["tables"], dt)
    k = np.asarray(p["tables"][0]).shape[1]
    z = flat.reshape(flat.shape[0], -1, k)
    inner = inner_product_layer(z, dt=dt)
    x = np.concatenate([flat, inner], axis=1)
    return dnn_layer(x, p["dnn_hidden"], p["dnn_out"], p.get("act", "relu"), dt=dt), x


def din(inputs, p, dense_feats, sparse_feats, behavior_feats, dt=np.float64,
        att_act="prelu", dnn_act="prelu"):
    """DIN.call (model/din.py:56-95).

    behavior_feats in sparse-column order (the reference builds history_seq
    and embed_seq_layers by iterating sparse_feature_columns, :44-46,73-78);
    inputs['movie_id'] is [B, n_behaviour] (candidate_item[:, i], :79).
    p: 'sparse_tables' {feat: table} for non-behaviour sparse feats,
       'seq_tables' {feat: table} for behaviour feats, 'att' attention params,
       'bn' (gamma, beta, mean, var, eps), 'dnn' [(kernel, bias, act_params)]
       with act_params = alpha [units] for dnn_act 'prelu' (Dense(unit,
       activation=PReLU()), :51) or (alpha, mean, var, eps) for 'dice'
       (Dense(unit, activation=Dice()), layer/interaction.py:410-425 at
       inference), 'out' (kernel, bias)."""
    dense_in = np.concatenate([cast_inputs(inputs[f], dt).reshape(-1, 1) for f in dense_feats], -1)
    other_sparse = [f for f in sparse_feats if f not in behavior_feats]
    sp = np.concatenate([np.asarray(inputs[f]).reshape(-1, 1) for f in other_sparse], -1)
    other = np.concatenate([embedding_lookup(np.asarray(p["sparse_tables"][f], dt), sp[:, i])
                            for i, f in enumerate(other_sparse)], -1)
    other = np.concatenate([other, dense_in], -1)
    hist = np.stack([np.asarray(inputs[f]) for f in behavior_feats], -1)  # [B,T,nb]
    cand = np.asarray(inputs["movie_id"]).reshape(hist.shape[0], -1)
    seq = np.concatenate([embedding_lookup(np.asarray(p["seq_tables"][f], dt), hist[:, :, i])
                          for i, f in enumerate(behavior_feats)], -1)
    item = np.concatenate([embedding_lookup(np.asarray(p["seq_tables"][f], dt), cand[:, i])
                           for i, f in enumerate(behavior_feats)], -1)
    mask = (hist[:, :, 0] != 0).astype(dt)
    att = attention(item, seq, seq, mask, p["att"], att_act, dt=dt)
    emb = np.concatenate([att, item, other], -1)
    g, bt, mu, var, eps = p["bn"]
    emb = batchnorm_inference(emb, mu, var, g, bt, eps, dt=dt)
    for kern, bias, ap in p["dnn"]:
        if dnn_act == "prelu":
            emb = dense(emb, kern, bias, "prelu", ap, dt=dt)
        elif dnn_act == "dice":
            alpha, dmu, dvar, deps = ap
            emb = dice(dense(emb, kern, bias, None, dt=dt), alpha, dmu, dvar, deps, dt=dt)
        else:
            raise ValueError(dnn_act)
    return sigmoid(dense(emb, p["out"][0], p["out"][1], dt=dt)), att


# ------------------------------------ other interactions
def interaction_layer(e, dt=np.float64):
    """InteractionLayer.call (layer/interaction.py:286-297): [B,F,k] ->
    [B,P,k] element-wise products of the (i<j) row-major pairs."""
    e = np.asarray(e, dt)
    prods = [e[:, i] * e[:, j] for i in range(e.shape[1]) for j in range(i + 1, e.shape[1])]
    return np.transpose(np.asarray(prods), (1, 0, 2))


def attention_layer(x, p, dt=np.float64):
    """AttentionLayer.call (layer/interaction.py:310-319) op for op:
    Dense(P, relu) -> Dense(1) -> tf.nn.softmax over the LAST axis (size 1:
    every score is exactly 1) -> transpose -> matmul with the inputs."""
    x = np.asarray(x, dt)
    h = activation(np.tensordot(x, np.asarray(p["att_w_kernel"], dt), axes=1) + np.asarray(p["att_w_bias"], dt),
                   "relu")
    s = np.tensordot(h, np.asarray(p["att_h_kernel"], dt), axes=1) + np.asarray(p["att_h_bias"], dt)  # [B,P,1]
    e = np.exp(s - s.max(axis=-1, keepdims=True))
    a = e / e.sum(axis=-1, keepdims=True)                                     # softmax over axis -1
    a = np.transpose(a, (0, 2, 1))                                            # [B,1,P]
    return np.matmul(a, x).reshape(-1, x.shape[2])


def afm(X, p, mode, nd=13, dt=np.float64, inputs=None):
    """AFM.call (model/afm.py:15-19) over AFMLayer.call
    (layer/interaction.py:333-351): per-field Embedding(feat_onehot_dim,
    embed_dim) -> [B,F,k] -> InteractionLayer -> mean / max / attention over
    the pairs -> Dense(1) -> sigmoid, then AFM's second sigmoid."""
    _, sparse = inputs if inputs is not None else _split_dense_sparse(X, nd, dt)
    sparse = np.asarray(sparse)
    embed = np.transpose(np.stack([embedding_lookup(np.asarray(t, dt), sparse[:, i])
                                   for i, t in enumerate(p["tables"])], 0), (1, 0, 2))
    pairs = interaction_layer(embed, dt)
    if mode == "avg":
        x = np.mean(pairs, axis=1)
    elif mode == "max":
        x = np.max(pairs, axis=1)
    else:
        x = attention_layer(pairs, p, dt)
    out = sigmoid(dense(x, p["out_kernel"], p["out_bias"], dt=dt))
    return sigmoid(out), x


def bi_interaction(e, dt=np.float64):
    """NFM's Bi-Interaction (model/nfm.py:28) on a 3-D embedding [B,F,k]:
    0.5 * (sum_f e)^2 - sum_f e^2, per dim -> [B,k]."""
    e = np.asarray(e, dt)
    return 0.5 * (np.power(np.sum(e, axis=1), 2) - np.sum(np.power(e, 2), axis=1))


def nfm(X, p, nd=13, dt=np.float64, inputs=None):
    """NFM.call (model/nfm.py:22-33) with 3-D embeddings (documented
    deviation: on the reference's rank-2 EmbedLayer output the reduce_sum over
    axis 1 yields [B] and the concat with the dense block fails):
    x = BN(concat([dense, BiInteraction(emb)])) -> DNNLayer -> Dense(1) -> sigmoid."""
    dense_in, sparse = inputs if inputs is not None else _split_dense_sparse(X, nd, dt)
    flat = embed_layer(sparse, p["tables"], dt)
    k = np.asarray(p["tables"][0]).shape[1]
    emb = bi_interaction(flat.reshape(flat.shape[0], -1, k), dt)
    x = np.concatenate([np.asarray(dense_in, dt), emb], axis=-1)
    x = batchnorm_inference(x, p["bn_mean"], p["bn_var"], p.get("bn_gamma"), p.get("bn_beta"), dt=dt)
    x = dnn_layer(x, p["dnn_hidden"], p["dnn_out"], p.get("act", "relu"), dt=dt)
    return sigmoid(dense(x, p["out_kernel"], p["out_bias"], dt=dt)), emb


def ffm_layer(dense_in, sparse, onehot_dims, w0, w, v, dt=np.float64):
    """FFMLayer.call (layer/interaction.py:134-163) op for op: x = [dense |
    one_hot(id_c, feat_onehot_dim_c) ...]; linear = w0 + x@w; field_f =
    tensordot(x, v) [B, NF, k]; inter = sum_{i<j} sum(field_f[:,i] *
    field_f[:,j]).  Builds the dense one-hot matrix: small vocabularies only."""
    dense_in = np.asarray(dense_in, dt)
    ids = cast_ids(sparse)
    B = dense_in.shape[0]
    parts = [dense_in]
    for c, depth in enumerate(onehot_dims):
        col = ids[:, c]
        oh = np.zeros((B, depth), dt)
        ok = (col >= 0) & (col < depth)  # tf.one_hot: out-of-range -> zero row
        oh[np.nonzero(ok)[0], col[ok]] = 1.0
        parts.append(oh)
    x = np.concatenate(parts, axis=1)
    linear = np.asarray(w0, dt) + x @ np.asarray(w, dt)
    field_f = np.tensordot(x, np.asarray(v, dt), axes=1)
    inter = np.zeros((B, 1), dt)
    NF = field_f.shape[1]
    for i in range(NF):
        for j in range(i + 1, NF):
            inter += np.sum(field_f[:, i] * field_f[:, j], axis=1, keepdims=True)
    return linear + inter


def ffm_layer_gather(dense_in, sparse, onehot_dims, w0, w, v, dt=np.float64):
    """ffm_layer without the one-hot matrix (for vocabularies too large to
    materialise, e.g. the bench's 26 x 1e6 CPU baseline): x has exactly one 1
    per field at column nd + offset_c + id_c, so x@w and tensordot(x, v) are
    row gathers (pinned == ffm_layer by tests/test_interactions.py);
    out-of-range ids contribute a zero row like tf.one_hot."""
    dense_in = np.asarray(dense_in, dt)
    ids = cast_ids(sparse)
    nd = dense_in.shape[1]
    w, v = np.asarray(w), np.asarray(v)
    offs = np.concatenate([[0], np.cumsum(onehot_dims)[:-1]]).astype(np.int64)
    ok = (ids >= 0) & (ids < np.asarray(onehot_dims)[None, :])
    rows = np.where(ok, nd + offs[None, :] + ids, 0)
    okf = ok.astype(dt)
    Fm = np.einsum("bi,ifk->bfk", dense_in, v[:nd].astype(dt)) + np.einsum("bc,bcfk->bfk", okf, v[rows].astype(dt))
    lin = np.asarray(w0, dt) + dense_in @ w[:nd].astype(dt) + (okf * w[rows, 0].astype(dt)).sum(1, keepdims=True)
    inter = dt(0.5) * ((Fm.sum(1) ** 2).sum(1) - (Fm ** 2).sum((1, 2)))
    return lin + inter[:, None]


def ffm(X, p, onehot_dims, nd=13, dt=np.float64, inputs=None):
    """FFM.call (model/ffm.py:20-22): sigmoid(FFMLayer(inputs))."""
    dense_in, sparse = inputs if inputs is not None else _split_dense_sparse(X, nd, dt)
    return sigmoid(ffm_layer(dense_in, sparse, onehot_dims, p["w0"], p["w"], p["v"], dt=dt))


# --------------------------------------------- training
def onehot_matrix(dense, ids, field_vocab, dt=np.float64):
    """utils/dataset.py:47-48 (pd.get_dummies): x = [dense | one-hot per
    field], field c's block starts at nd + sum(vocab[:c])."""
    dense = np.asarray(dense, dt)
    ids = cast_ids(ids)
    offs = np.concatenate([[0], np.cumsum(field_vocab)[:-1]]).astype(np.int64)
    B, nd = dense.shape
    x = np.zeros((B, nd + int(np.sum(field_vocab))), dt)
    x[:, :nd] = dense
    x[np.arange(B)[:, None], nd + offs[None, :] + ids] = 1.0
    return x


def fm_loss(x, t, w0, w1, v, l2_w, l2_v, dt=np.float64):
    """compile_fit's objective for FM (utils/compile_fit.py:9-15,
    model/fm.py:19-23): mean binary cross-entropy of sigmoid(FMLayer(x))
    (Keras takes the sigmoid's logits: softplus form) + l2_w |w1|^2 + l2_v |v|^2."""
    y = fm_layer(x, w0, w1, v, dt)[:, 0]
    t = np.asarray(t, dt)
    ce = np.maximum(y, 0) - y * t + np.log1p(np.exp(-np.abs(y)))
    return np.mean(ce) + l2_w * np.sum(np.asarray(w1, dt) ** 2) + l2_v * np.sum(np.asarray(v, dt) ** 2), ce


def fm_train_step(x, t, w0, w1, v, lr, l2_w, l2_v, dt=np.float64):
    """One SGD step (tf.keras SGD: w -= lr * dL/dw) of fm_loss, gradients in
    closed form: g = (sigmoid(y) - t)/B, dL/dw0 = sum g, dL/dw1 = x^T g +
    2 l2_w w1, dL/dv = x^T (g * s) - (x^2)^T g * v + 2 l2_v v, s = x @ v.
    Returns (w0, w1, v) after the step and the per-sample losses before it."""
    x = np.asarray(x, dt)
    w0, w1, v = (np.asarray(a, dt) for a in (w0, w1, v))
    y = fm_layer(x, w0, w1, v, dt)[:, 0]
    t = np.asarray(t, dt)
    g = (sigmoid(y) - t) / x.shape[0]
    s = x @ v
    g_w0 = np.sum(g, keepdims=True)
    g_w1 = x.T @ g[:, None] + 2 * l2_w * w1
    g_v = x.T @ (g[:, None] * s) - ((x * x).T @ g)[:, None] * v + 2 * l2_v * v
    ce = np.maximum(y, 0) - y * t + np.log1p(np.exp(-np.abs(y)))
    return w0 - lr * g_w0, w1 - lr * g_w1, v - lr * g_v, ce


def ffm_loss(dense, ids, t, w0, w, v, onehot_dims, l2_w, l2_v, dt=np.float64):
    """compile_fit's objective on FFM (model/ffm.py:20-22): mean BCE of
    sigmoid(FFMLayer) plus FFMLayer's l2(w_reg) on w and l2(v_reg) on v
    (layer/interaction.py:131-139; Keras fit adds model.losses)."""
    z = ffm_layer(dense, ids, onehot_dims, w0, w, v, dt)[:, 0]
    t = np.asarray(t, dt).reshape(-1)
    bce = np.mean(np.maximum(z, 0) - z * t + np.log1p(np.exp(-np.abs(z))))
    return bce + l2_w * np.sum(np.asarray(w, dt) ** 2) + l2_v * np.sum(np.asarray(v, dt) ** 2)


def ffm_train_step(dense, ids, t, w0, w, v, onehot_dims, lr, l2_w, l2_v, dt=np.float64):
    """One SGD step of ffm_loss in closed form: with x the one-hot input,
    Fm_f = sum_i x_i v[i, f] and inter = 0.5 (|sum_f Fm_f|^2 - sum_f |Fm_f|^2),
    g = (sigmoid(z) - t)/B and G_b[f] = g_b (T_b - Fm_bf), T = sum_f Fm_f:
    dw0 = sum g, dw = x^T g + 2 l2_w w, dv[i, f] = sum_b x_bi G_b[f] + 2 l2_v v.
    Returns ((w0, w, v) after the step, per-sample BCE losses before it)."""
    x = onehot_matrix(dense, ids, onehot_dims, dt)
    w0, w, v = (np.asarray(a, dt) for a in (w0, w, v))
    Fm = np.tensordot(x, v, axes=1)                          # [B, NF, k]
    T = Fm.sum(1, keepdims=True)
    z = (w0 + x @ w)[:, 0] + 0.5 * ((T[:, 0] ** 2).sum(1) - (Fm ** 2).sum((1, 2)))
    t = np.asarray(t, dt).reshape(-1)
    loss = np.maximum(z, 0) - z * t + np.log1p(np.exp(-np.abs(z)))
    g = (sigmoid(z) - t) / z.shape[0]
    G = g[:, None, None] * (T - Fm)
    dv = np.tensordot(x, G, axes=[[0], [0]]) + 2 * l2_v * v
    dw = x.T @ g[:, None] + 2 * l2_w * w
    return (w0 - lr * g.sum(keepdims=True)[:1], w - lr * dw, v - lr * dv), loss


def _dnn_train_acts(x, layers, act, masks, dt):
    """DNNLayer.call in training (layer/interaction.py:40-46): Dense +
    activation, then Dropout (masks[i] or the identity) per hidden layer."""
    acts = [x]
    for i, (W, b) in enumerate(layers[:-1]):
        a = activation(acts[-1] @ W + b, act)
        acts.append(a * np.asarray(masks[i], dt) if masks is not None else a)
    return acts


def _dnn_train_bwd(delta, layers, acts, act, masks, lr):
    """Backward of _dnn_train_acts + the output Dense: returns the SGD-updated
    layers and dL/dx.  Through hidden layer i: ReLU' = [a > 0] (a after the
    dropout: zero where dropped) and the dropout multiplier masks[i]."""
    new_layers = [None] * len(layers)
    for li in reversed(range(len(layers))):
        W, b = layers[li]
        dW, db = acts[li].T @ delta, delta.sum(0)
        prev = delta @ W.T
        if li > 0 and act == "relu":
            prev = prev * (acts[li] > 0)
        if li > 0 and masks is not None:
            prev = prev * np.asarray(masks[li - 1], prev.dtype)
        new_layers[li] = (W - lr * dW, b - lr * db)
        delta = prev
    return new_layers, delta


_PHILOX_M = (np.uint64(0xD2511F53), np.uint64(0xCD9E8D57))
_PHILOX_W = (np.uint32(0x9E3779B9), np.uint32(0xBB67AE85))


def philox4x32_10(ctr, seed):
    """Philox4x32-10 (Salmon et al., SC'11) on counters ctr (uint64 array,
    words (lo, hi, 0, 0)) with the 64-bit key seed: returns [n, 4] uint32."""
    ctr = np.asarray(ctr, np.uint64)
    c = [(ctr & np.uint64(0xFFFFFFFF)).astype(np.uint32), (ctr >> np.uint64(32)).astype(np.uint32),
         np.zeros(ctr.shape, np.uint32), np.zeros(ctr.shape, np.uint32)]
    k0, k1 = np.uint32(seed & 0xFFFFFFFF), np.uint32((seed >> 32) & 0xFFFFFFFF)
    with np.errstate(over="ignore"):
        for _ in range(10):
            p0 = _PHILOX_M[0] * c[0].astype(np.uint64)
            p1 = _PHILOX_M[1] * c[2].astype(np.uint64)
            c = [(p1 >> np.uint64(32)).astype(np.uint32) ^ c[1] ^ k0, (p1 & np.uint64(0xFFFFFFFF)).astype(np.uint32),
                 (p0 >> np.uint64(32)).astype(np.uint32) ^ c[3] ^ k1, (p0 & np.uint64(0xFFFFFFFF)).astype(np.uint32)]
            k0 = np.uint32(k0 + _PHILOX_W[0])
            k1 = np.uint32(k1 + _PHILOX_W[1])
    return np.stack(c, axis=-1)


def dropout_multiplier(rows, cols, rate, seed, offset, dt=np.float64):
    """DNNLayer's Dropout(rate) in training (layer/interaction.py:35,44;
    tf.nn.dropout: keep = u >= rate, kept values scaled by 1/(1-rate)) with
    the build's counter-based draws (rs_dropout): element e = row*cols + col
    takes word (offset+e) % 4 of Philox4x32-10(counter (offset+e)//4, key
    seed), u = (word >> 8) 2^-24.  Returns the [rows, cols] multiplier
    keep / (1 - rate) (the fp32 scale, as the kernel applies it)."""
    e = np.uint64(offset) + np.arange(rows * cols, dtype=np.uint64)
    words = philox4x32_10(e >> np.uint64(2), int(seed))
    w = words[np.arange(e.size), (e & np.uint64(3)).astype(np.int64)]
    u = (w >> np.uint32(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)
    scale = np.float32(1.0) / (np.float32(1.0) - np.float32(rate))
    return np.where(u >= np.float32(rate), scale, np.float32(0.0)).astype(dt).reshape(rows, cols)


def deepfm_train_step(dense, ids, t, p, lr, l2_w, l2_v, nd=13, act="relu", dt=np.float64, masks=None):
    """One SGD step of compile_fit on DeepFM (model/deepFM.py:23-31,
    utils/compile_fit.py:9-15), backpropagated by hand: z = 0.5 (fm + dnn),
    g = (sigmoid(z) - t)/B; DNN layers by the chain rule (ReLU' = [a > 0]);
    FM w.r.t. x: w1 + v s - x |v|^2 per feature; w1 / v with their l2
    terms; embedding rows by scatter-add (np.add.at) of dL/dx's sparse block.
    p: {"tables", "w0", "w1", "v", "dnn_hidden": [(W, b)], "dnn_out": (W, b)}.
    masks: DNNLayer's Dropout in training — per hidden layer the [B, h]
    multiplier keep / (1 - rate) applied after its activation (and to the
    gradient flowing back through it), or None (Dropout as the identity).
    Returns (new p, per-sample losses before the step)."""
    dense = np.asarray(dense, dt)
    ids = cast_ids(ids)
    t = np.asarray(t, dt)
    tables = [np.array(tb, dt) for tb in p["tables"]]
    k = tables[0].shape[1]
    x = np.concatenate([dense, embed_layer(ids, tables, dt)], axis=1)
    w0, w1, v = (np.array(p[n], dt) for n in ("w0", "w1", "v"))
    layers = [(np.array(W, dt), np.array(b, dt)) for W, b in p["dnn_hidden"]] + \
             [(np.array(p["dnn_out"][0], dt), np.array(p["dnn_out"][1], dt))]
    acts = _dnn_train_acts(x, layers, act, masks, dt)
    dnn = (acts[-1] @ layers[-1][0] + layers[-1][1])[:, 0]
    fm = fm_layer(x, w0, w1, v, dt)[:, 0]
    z = 0.5 * (fm + dnn)
    g = (sigmoid(z) - t) / x.shape[0]
    gf = gd = 0.5 * g
    loss = np.maximum(z, 0) - z * t + np.log1p(np.exp(-np.abs(z)))
    new_layers, delta = _dnn_train_bwd(gd[:, None], layers, acts, act, masks, lr)
    s = x @ v
    dx = delta + gf[:, None] * (w1[:, 0][None, :] + s @ v.T - x * np.sum(v * v, axis=1)[None, :])
    dw1 = x.T @ gf[:, None]
    dv = x.T @ (gf[:, None] * s) - ((x * x).T @ gf)[:, None] * v
    out = {"w0": w0 - lr * gf.sum(keepdims=True), "w1": w1 - lr * (dw1 + 2 * l2_w * w1),
           "v": v - lr * (dv + 2 * l2_v * v), "dnn_hidden": new_layers[:-1], "dnn_out": new_layers[-1]}
    for c, tb in enumerate(tables):
        np.add.at(tb, ids[:, c], -lr * dx[:, nd + c * k: nd + (c + 1) * k])
    out["tables"] = tables
    return out, loss


KERAS_EPS = 1e-7  # keras.backend.epsilon()


def pnn_bce(pre, t, dt=np.float64):
    """model/pnn.py:79: tf.reduce_mean(losses.binary_crossentropy(y_train,
    pre)) with y_train [B] and pre = the DNN LOGIT [B, 1] (no sigmoid).
    Keras' probability form clips pre to [eps, 1-eps] and adds eps inside the
    logs; the [B] labels broadcast against [B, 1] to [B, B] before the mean
    over the last axis, so sample i's loss is the mean over j of
    BCE(y_j, pre_i) = -(ybar log(q_i + eps) + (1 - ybar) log(1 - q_i + eps)).
    Returns (mean loss, per-sample losses)."""
    pre = np.asarray(pre, dt).reshape(-1)
    t = np.asarray(t, dt).reshape(-1)
    q = np.clip(pre, KERAS_EPS, 1 - KERAS_EPS)
    per = -(t[None, :] * np.log(q[:, None] + KERAS_EPS) + (1 - t[None, :]) * np.log(1 - q[:, None] + KERAS_EPS))
    per = per.mean(axis=1)
    return per.mean(), per


def _pnn_x(e, flat, p, mode, dt):
    parts = [flat]
    if mode in ("inner", "both"):
        parts.append(inner_product_layer(e, dt=dt))
    if mode in ("outer", "both"):
        parts.append(outer_product_layer(e, p["outer_W"], dt=dt))
    return np.concatenate(parts, axis=1)


def pnn_train_step(ids, t, p, lr, act="relu", dt=np.float64, mode="inner"):
    """One step of the reference's PNN loop (model/pnn.py:74-81: GradientTape,
    SGD(lr) over model.variables) for mode 'inner' / 'outer' / 'both' (the
    loop's own example runs 'both', :61), backpropagated by hand:
    dL/dpre_i = (-ybar/(q_i+eps) + (1-ybar)/(1-q_i+eps))/B inside the clip
    range, 0 outside (tf.clip_by_value); the DNN by the chain rule (Dropout is
    the identity: the loop calls model(X) without training=True); the inner
    products p_ij = e_i . e_j give de_i += dL/dp_ij e_j; the outer products
    o_p = e_j^T W_p e_i (W_p[a][c] = W[a,p,c], i = row(p), j = col(p),
    layer/interaction.py:200-215) give de_i += g_p W_p^T e_j, de_j += g_p W_p e_i
    and dW[a,p,c] = sum_b g_bp e_j[a] e_i[c]; embedding rows by scatter-add.
    No regularisers: the loop's loss is the BCE alone (OuterProductLayer's
    l2(1e-4) sits in model.losses, which the loop never adds).
    Returns (new p, per-sample losses before the step)."""
    ids = cast_ids(ids)
    t = np.asarray(t, dt).reshape(-1)
    tables = [np.array(tb, dt) for tb in p["tables"]]
    k = tables[0].shape[1]
    F = len(tables)
    flat = embed_layer(ids, tables, dt)
    e = flat.reshape(flat.shape[0], F, k)
    x = _pnn_x(e, flat, p, mode, dt)
    layers = [(np.array(W, dt), np.array(b, dt)) for W, b in p["dnn_hidden"]] + \
             [(np.array(p["dnn_out"][0], dt), np.array(p["dnn_out"][1], dt))]
    acts = [x]
    for W, b in layers[:-1]:
        acts.append(activation(acts[-1] @ W + b, act))
    pre = (acts[-1] @ layers[-1][0] + layers[-1][1])[:, 0]
    _, loss = pnn_bce(pre, t, dt)
    B = x.shape[0]
    ybar = t.mean()
    q = np.clip(pre, KERAS_EPS, 1 - KERAS_EPS)
    inside = (pre >= KERAS_EPS) & (pre <= 1 - KERAS_EPS)
    g = np.where(inside, (-ybar / (q + KERAS_EPS) + (1 - ybar) / (1 - q + KERAS_EPS)) / B, 0.0)
    delta = g[:, None]
    new_layers = [None] * len(layers)
    for li in reversed(range(len(layers))):
        W, b = layers[li]
        dW, db = acts[li].T @ delta, delta.sum(0)
        prev = delta @ W.T
        if li > 0 and act == "relu":
            prev = prev * (acts[li] > 0)
        new_layers[li] = (W - lr * dW, b - lr * db)
        delta = prev
    de = delta[:, :F * k].reshape(B, F, k).copy()
    row, col = pair_indices(F)
    P = len(row)
    off = F * k
    new = {}
    if mode in ("inner", "both"):
        dpi = delta[:, off:off + P]
        off += P
        for pi, (i, j) in enumerate(zip(row, col)):
            de[:, i, :] += dpi[:, pi:pi + 1] * e[:, j, :]
            de[:, j, :] += dpi[:, pi:pi + 1] * e[:, i, :]
    if mode in ("outer", "both"):
        W = np.array(p["outer_W"], dt)  # [k, P, k]
        dpo = delta[:, off:off + P]
        dW = np.zeros_like(W)
        for pi, (i, j) in enumerate(zip(row, col)):
            Wp = W[:, pi, :]                                      # [a, c]
            g = dpo[:, pi:pi + 1]
            de[:, i, :] += g * (e[:, j, :] @ Wp)                  # sum_a e_j[a] W[a,c]
            de[:, j, :] += g * (e[:, i, :] @ Wp.T)                # sum_c W[a,c] e_i[c]
            dW[:, pi, :] = (g * e[:, j, :]).T @ e[:, i, :]        # sum_b g e_j[a] e_i[c]
        new["outer_W"] = W - lr * dW
    for c, tb in enumerate(tables):
        np.add.at(tb, ids[:, c], -lr * de[:, c, :])
    new.update({"tables": tables, "dnn_hidden": new_layers[:-1], "dnn_out": new_layers[-1]})
    return new, loss


def pnn_loss(ids, t, p, act="relu", dt=np.float64, mode="inner"):
    """The PNN loop's objective (pnn_bce of the forward in ``mode``)."""
    flat = embed_layer(cast_ids(ids), p["tables"], dt)
    k = np.asarray(p["tables"][0]).shape[1]
    e = flat.reshape(flat.shape[0], -1, k)
    x = _pnn_x(e, flat, p, mode, dt)
    pre = dnn_layer(x, p["dnn_hidden"], p["dnn_out"], act, dt)
    return pnn_bce(pre, t, dt)[0]


def _dice_train(z, alpha, eps, dt):
    """Dice.call in training (layer/interaction.py:416-425 under fit): its
    BatchNormalization(center=False, scale=False) normalises with the batch's
    mean and biased variance over every axis but the last."""
    axes = tuple(range(z.ndim - 1))
    mu, var = z.mean(axes), z.var(axes)
    zh = (z - mu) / np.sqrt(var + eps)
    pz = 1.0 / (1.0 + np.exp(-zh))
    a = np.asarray(alpha, dt)
    return a * (1.0 - pz) * z + pz * z, (mu, var, zh, pz)


def _dice_train_bwd(dy, z, alpha, eps, saved):
    """dL/dz and dL/dalpha of _dice_train: y = alpha (1-p) z + p z, p =
    sigmoid(zhat); through zhat the batch-norm backward without gamma."""
    mu, var, zh, pz = saved
    axes = tuple(range(z.ndim - 1))
    a = np.asarray(alpha, dy.dtype)
    dalpha = (dy * (1.0 - pz) * z).sum(axes)
    dx = dy * (a * (1.0 - pz) + pz)
    dzh = dy * (1.0 - a) * z * pz * (1.0 - pz)
    dx = dx + (dzh - dzh.mean(axes) - zh * (dzh * zh).mean(axes)) / np.sqrt(var + eps)
    return dx, dalpha


def _din_train_forward(inputs, p, dense_feats, sparse_feats, behavior_feats, dt, att_act="prelu", dnn_act="prelu",
                       drop_mask=None):
    """DIN.call (model/din.py:56-95) with training=True (Keras fit): the
    BatchNormalization normalises with the batch's own mean and (biased)
    variance, and so do the Dice layers' BatchNormalizations (the fit's
    training flag reaches every nested layer call).  att / dnn activation
    'prelu' (the reference defaults) or 'dice'.  Returns every intermediate
    the hand backward needs.  drop_mask: the Dropout after the DNN
    (model/din.py:93) as a fixed [B, h] multiplier, or None (the identity)."""
    c = {}
    dense_in = np.concatenate([cast_inputs(inputs[f], dt).reshape(-1, 1) for f in dense_feats], -1) \
        if dense_feats else None
    other_sparse = [f for f in sparse_feats if f not in behavior_feats]
    c["other_ids"] = [np.asarray(inputs[f]).reshape(-1) for f in other_sparse]
    parts = [embedding_lookup(np.asarray(p["sparse_tables"][f], dt), i) for f, i in zip(other_sparse, c["other_ids"])]
    if dense_in is not None:
        parts.append(dense_in)
    other = np.concatenate(parts, -1) if parts else None
    hist = np.stack([np.asarray(inputs[f]) for f in behavior_feats], -1)  # [B,T,nb]
    cand = np.asarray(inputs["movie_id"]).reshape(hist.shape[0], -1)
    c["hist"], c["cand"] = hist, cand
    seq = np.concatenate([embedding_lookup(np.asarray(p["seq_tables"][f], dt), hist[:, :, i])
                          for i, f in enumerate(behavior_feats)], -1)
    item = np.concatenate([embedding_lookup(np.asarray(p["seq_tables"][f], dt), cand[:, i])
                           for i, f in enumerate(behavior_feats)], -1)
    mask = hist[:, :, 0] != 0
    B, T, K = seq.shape
    q = np.tile(item[:, None, :], (1, T, 1))
    h = np.concatenate([q, seq, q - seq, q * seq], -1)
    att_pre, att_in = [], [h]
    if att_act == "prelu":
        for W, b, a in p["att"]["prelu"]:
            z = np.tensordot(att_in[-1], np.asarray(W, dt), axes=[[2], [0]]) + np.asarray(b, dt)
            att_pre.append(z)
            att_in.append(prelu(z, np.asarray(a, dt)))
    else:  # 'dice': len(hidden_units) Dice layers on the 4k-wide concat, no Dense (:363-364)
        for alpha, _, _, eps in p["att"]["dice"]:
            y, saved = _dice_train(att_in[-1], alpha, eps, dt)
            att_pre.append(saved)
            att_in.append(y)
    score = (np.tensordot(att_in[-1], np.asarray(p["att"]["out"][0], dt), axes=[[2], [0]])
             + np.asarray(p["att"]["out"][1], dt))[..., 0]
    score = np.where(mask, score, dt(np.float32(MASK_FILL)))
    e = np.exp(score - score.max(-1, keepdims=True))
    a = e / e.sum(-1, keepdims=True)
    att = np.einsum("bt,btk->bk", a, seq)
    x = np.concatenate([att, item] + ([other] if other is not None else []), -1)
    g, bt, mu, var, eps = p["bn"]
    bmu, bvar = x.mean(0), x.var(0)
    xhat = (x - bmu) / np.sqrt(bvar + eps)
    y = xhat * np.asarray(g, dt) + np.asarray(bt, dt)
    pre, acts, dsaved = [], [y], []
    for W, b, al in p["dnn"]:
        z = acts[-1] @ np.asarray(W, dt) + np.asarray(b, dt)
        pre.append(z)
        if dnn_act == "prelu":
            acts.append(prelu(z, np.asarray(al, dt)))
        else:
            yz, saved = _dice_train(z, al[0], al[3], dt)
            dsaved.append(saved)
            acts.append(yz)
    top = acts[-1] * np.asarray(drop_mask, dt) if drop_mask is not None else acts[-1]
    logit = (top @ np.asarray(p["out"][0], dt) + np.asarray(p["out"][1], dt))[:, 0]
    c.update(top=top, seq=seq, item=item, mask=mask, q=q, att_pre=att_pre, att_in=att_in, a=a, x=x, bmu=bmu, bvar=bvar,
             xhat=xhat, pre=pre, acts=acts, dsaved=dsaved, logit=logit, B=B, T=T, K=K, nd=0 if dense_in is None else
             dense_in.shape[1], other_sparse=other_sparse)
    return c


def din_loss(inputs, t, p, dense_feats, sparse_feats, behavior_feats, dt=np.float64, att_act="prelu",
             dnn_act="prelu", drop_mask=None):
    """compile_fit's objective on DIN (training-mode forward): mean BCE."""
    z = _din_train_forward(inputs, p, dense_feats, sparse_feats, behavior_feats, dt, att_act, dnn_act,
                           drop_mask)["logit"]
    t = np.asarray(t, dt).reshape(-1)
    return np.mean(np.maximum(z, 0) - z * t + np.log1p(np.exp(-np.abs(z))))


def din_train_step(inputs, t, p, dense_feats, sparse_feats, behavior_feats, lr, momentum=0.99, dt=np.float64,
                   att_act="prelu", dnn_act="prelu", drop_mask=None):
    """One SGD step of compile_fit on DIN (utils/compile_fit.py:9-15; model/
    din.py:56-95, att 'prelu', dnn 'prelu'), backpropagated by hand:
    BCE on the sigmoid's logit (g = (sigmoid(z) - t)/B); Dense + PReLU layers
    (dalpha = sum dy min(0, z), the attention's alpha [T, h] summed over the
    batch); BatchNormalization in training mode (batch mean / biased variance,
    dx = gamma/sigma (dy - mean dy - xhat mean(dy xhat))) and its moving
    averages (momentum 0.99, biased batch variance); the masked softmax pool
    (ds_t = a_t (dv.seq_t - sum_s a_s dv.seq_s)); the [q, k, q-k, q*k] concat
    (dq sums over T); embedding rows by scatter-add.  No regularisers.
    Dice (att / dnn 'dice'): training-mode batch statistics in the forward,
    the batch-norm backward inside its gradient, its moving averages moved
    like the BN's.  drop_mask: the Dropout after the DNN (din.py:93) as a
    fixed [B, h] multiplier (dL/d(dnn out) = dL/d(dropped) * mask), or None.
    Returns (new p, per-sample losses before the step)."""
    c = _din_train_forward(inputs, p, dense_feats, sparse_feats, behavior_feats, dt, att_act, dnn_act, drop_mask)
    B, T, K = c["B"], c["T"], c["K"]
    t = np.asarray(t, dt).reshape(-1)
    z = c["logit"]
    loss = np.maximum(z, 0) - z * t + np.log1p(np.exp(-np.abs(z)))
    g = (sigmoid(z) - t) / B
    new = {"sparse_tables": {f: np.array(v, dt) for f, v in p["sparse_tables"].items()},
           "seq_tables": {f: np.array(v, dt) for f, v in p["seq_tables"].items()}}
    Wo, bo = (np.asarray(v, dt) for v in p["out"])
    new["out"] = (Wo - lr * (c["top"].T @ g[:, None]), bo - lr * g.sum(keepdims=True))
    dh = g[:, None] @ Wo.T
    if drop_mask is not None:
        dh = dh * np.asarray(drop_mask, dt)
    new_dnn = [None] * len(p["dnn"])
    for li in reversed(range(len(p["dnn"]))):
        W, b = (np.asarray(v, dt) for v in p["dnn"][li][:2])
        zl = c["pre"][li]
        if dnn_act == "prelu":
            al = np.asarray(p["dnn"][li][2], dt)
            dz = dh * np.where(zl > 0, 1.0, al)
            dal = (dh * np.minimum(zl, 0)).sum(0)
            ap_new = al - lr * dal
        else:
            al, dmu, dvar, deps = p["dnn"][li][2]
            dz, dal = _dice_train_bwd(dh, zl, al, deps, c["dsaved"][li])
            bmu_l, bvar_l = c["dsaved"][li][:2]
            ap_new = (np.asarray(al, dt) - lr * dal, momentum * np.asarray(dmu, dt) + (1 - momentum) * bmu_l,
                      momentum * np.asarray(dvar, dt) + (1 - momentum) * bvar_l, deps)
        new_dnn[li] = (W - lr * (c["acts"][li].T @ dz), b - lr * dz.sum(0), ap_new)
        dh = dz @ W.T
    new["dnn"] = new_dnn
    gam, bet, mu, var, eps = p["bn"]
    gam, bet = np.asarray(gam, dt), np.asarray(bet, dt)
    xhat = c["xhat"]
    dgam, dbet = (dh * xhat).sum(0), dh.sum(0)
    inv = 1.0 / np.sqrt(c["bvar"] + eps)
    dx = gam * inv * (dh - dh.mean(0) - xhat * (dh * xhat).mean(0))
    new["bn"] = (gam - lr * dgam, bet - lr * dbet, momentum * np.asarray(mu, dt) + (1 - momentum) * c["bmu"],
                 momentum * np.asarray(var, dt) + (1 - momentum) * c["bvar"], eps)
    datt, ditem, doth = dx[:, :K], dx[:, K:2 * K], dx[:, 2 * K:]
    seq, a, mask = c["seq"], c["a"], c["mask"]
    da = np.einsum("bk,btk->bt", datt, seq)
    dseq = a[:, :, None] * datt[:, None, :]
    ds = a * (da - (a * da).sum(-1, keepdims=True))
    ds = np.where(mask, ds, 0.0)
    Wso, bso = (np.asarray(v, dt) for v in p["att"]["out"])
    hl = c["att_in"][-1]
    new_att_out = (Wso - lr * np.tensordot(hl, ds, axes=[[0, 1], [0, 1]])[:, None], bso - lr * np.array([ds.sum()]))
    dh3 = ds[:, :, None] * Wso[:, 0][None, None, :]
    if att_act == "prelu":
        new_prelu = [None] * len(p["att"]["prelu"])
        for li in reversed(range(len(p["att"]["prelu"]))):
            W, b, al = (np.asarray(v, dt) for v in p["att"]["prelu"][li])
            zl = c["att_pre"][li]
            dz = dh3 * np.where(zl > 0, 1.0, al)
            dal = (dh3 * np.minimum(zl, 0)).sum(0)
            new_prelu[li] = (W - lr * np.tensordot(c["att_in"][li], dz, axes=[[0, 1], [0, 1]]),
                             b - lr * dz.sum((0, 1)), al - lr * dal)
            dh3 = np.tensordot(dz, W.T, axes=[[2], [0]])
        new["att"] = {"prelu": new_prelu, "out": new_att_out}
    else:
        new_dice = [None] * len(p["att"]["dice"])
        for li in reversed(range(len(p["att"]["dice"]))):
            al, dmu, dvar, deps = p["att"]["dice"][li]
            saved = c["att_pre"][li]
            dh3, dal = _dice_train_bwd(dh3, c["att_in"][li], al, deps, saved)
            new_dice[li] = (np.asarray(al, dt) - lr * dal, momentum * np.asarray(dmu, dt) + (1 - momentum) * saved[0],
                            momentum * np.asarray(dvar, dt) + (1 - momentum) * saved[1], deps)
        new["att"] = {"dice": new_dice, "out": new_att_out}
    d0, d1, d2, d3 = (dh3[..., i * K:(i + 1) * K] for i in range(4))
    q = c["q"]
    dq = (d0 + d2 + seq * d3).sum(1)
    dseq = dseq + d1 - d2 + q * d3
    ditem = ditem + dq
    col = 0
    for i, f in enumerate(behavior_feats):
        k = np.asarray(p["seq_tables"][f]).shape[1]
        tb = new["seq_tables"][f]
        np.add.at(tb, c["hist"][:, :, i].reshape(-1), -lr * dseq[:, :, col:col + k].reshape(-1, k))
        np.add.at(tb, c["cand"][:, i], -lr * ditem[:, col:col + k])
        col += k
    col = 0
    for f, ids in zip(c["other_sparse"], c["other_ids"]):
        k = np.asarray(p["sparse_tables"][f]).shape[1]
        np.add.at(new["sparse_tables"][f], ids, -lr * doth[:, col:col + k])
        col += k
    return new, loss


def _nfm_train_forward(dense, ids, p, dt, masks=None):
    tables = [np.asarray(tb, dt) for tb in p["tables"]]
    k = tables[0].shape[1]
    flat = embed_layer(cast_ids(ids), tables, dt)
    e = flat.reshape(flat.shape[0], -1, k)
    x = np.concatenate([np.asarray(dense, dt), bi_interaction(e, dt)], axis=-1)
    g_, b_, _, _, eps = p["bn"]
    mu, var = x.mean(0), x.var(0)
    xhat = (x - mu) / np.sqrt(var + eps)
    acts = [xhat * np.asarray(g_, dt) + np.asarray(b_, dt)]
    for i, (W, b) in enumerate(p["dnn_hidden"]):  # DNNLayer: Dense, then Dropout (masks[i] or the identity)
        a = activation(acts[-1] @ np.asarray(W, dt) + np.asarray(b, dt), p.get("act", "relu"))
        acts.append(a * np.asarray(masks[i], dt) if masks is not None else a)
    acts.append(acts[-1] @ np.asarray(p["dnn_out"][0], dt) + np.asarray(p["dnn_out"][1], dt))
    logit = (acts[-1] @ np.asarray(p["out"][0], dt) + np.asarray(p["out"][1], dt))[:, 0]
    return dict(e=e, x=x, mu=mu, var=var, xhat=xhat, acts=acts, logit=logit)


def nfm_loss(dense, ids, t, p, dt=np.float64, masks=None):
    """compile_fit's objective on NFM (training-mode BatchNormalization;
    masks: fixed dropout multipliers, or None)."""
    z = _nfm_train_forward(dense, ids, p, dt, masks)["logit"]
    t = np.asarray(t, dt).reshape(-1)
    return np.mean(np.maximum(z, 0) - z * t + np.log1p(np.exp(-np.abs(z))))


def nfm_train_step(dense, ids, t, p, lr, momentum=0.99, dt=np.float64, masks=None):
    """One SGD step of compile_fit on NFM (utils/compile_fit.py:9-15;
    model/nfm.py:22-33 with 3-D embeddings, training=True): BCE on the
    sigmoid's logit; output Dense(1) and the DNNLayer (relu hidden, linear
    output) by the chain rule; BatchNormalization in training mode (batch
    mean / biased variance, moving averages with momentum); the
    Bi-Interaction 0.5((sum_f e_f)^2 - sum_f e_f^2) gives de_f = dbi (S - e_f),
    S = sum_f e_f; embedding rows by scatter-add.  No regularisers.
    p: tables, bn (gamma, beta, mean, var, eps), dnn_hidden [(W, b)],
    dnn_out (W, b), out (W, b).  masks: DNNLayer's Dropout (interaction.py:
    44) in training, per hidden layer a [B, h] multiplier (None = the
    identity); the backward multiplies dL/d(hidden out) by it.
    Returns (new p, per-sample losses)."""
    ids = cast_ids(ids)
    c = _nfm_train_forward(dense, ids, p, dt, masks)
    t = np.asarray(t, dt).reshape(-1)
    z = c["logit"]
    B = z.shape[0]
    loss = np.maximum(z, 0) - z * t + np.log1p(np.exp(-np.abs(z)))
    g = (sigmoid(z) - t) / B
    layers = [(np.asarray(W, dt), np.asarray(b, dt)) for W, b in p["dnn_hidden"]]
    layers += [(np.asarray(p["dnn_out"][0], dt), np.asarray(p["dnn_out"][1], dt)),
               (np.asarray(p["out"][0], dt), np.asarray(p["out"][1], dt))]
    acts = c["acts"]
    nh = len(p["dnn_hidden"])
    delta = g[:, None]
    new_layers = [None] * len(layers)
    for li in reversed(range(len(layers))):
        W, b = layers[li]
        new_layers[li] = (W - lr * (acts[li].T @ delta), b - lr * delta.sum(0))
        prev = delta @ W.T
        if 0 < li <= nh and p.get("act", "relu") == "relu":  # acts[li] = relu output of hidden layer li-1
            prev = prev * (acts[li] > 0)
        if 0 < li <= nh and masks is not None:
            prev = prev * np.asarray(masks[li - 1], dt)
        delta = prev
    gam, bet, mu0, var0, eps = p["bn"]
    gam, bet = np.asarray(gam, dt), np.asarray(bet, dt)
    xhat = c["xhat"]
    dgam, dbet = (delta * xhat).sum(0), delta.sum(0)
    dx = gam / np.sqrt(c["var"] + eps) * (delta - delta.mean(0) - xhat * (delta * xhat).mean(0))
    nd = np.asarray(dense).shape[1]
    dbi = dx[:, nd:]
    e = c["e"]
    de = dbi[:, None, :] * (e.sum(1, keepdims=True) - e)
    tables = [np.array(tb, dt) for tb in p["tables"]]
    for f, tb in enumerate(tables):
        np.add.at(tb, ids[:, f], -lr * de[:, f, :])
    new = {"tables": tables, "dnn_hidden": new_layers[:nh], "dnn_out": new_layers[nh], "out": new_layers[nh + 1],
           "bn": (gam - lr * dgam, bet - lr * dbet, momentum * np.asarray(mu0, dt) + (1 - momentum) * c["mu"],
                  momentum * np.asarray(var0, dt) + (1 - momentum) * c["var"], eps)}
    if "act" in p:
        new["act"] = p["act"]
    return new, loss


def deepfm_loss(dense, ids, t, p, l2_w, l2_v, nd=13, dt=np.float64, masks=None):
    """compile_fit's objective on DeepFM: mean BCE(t, sigmoid(0.5(fm+dnn)))
    + l2_w |w1|^2 + l2_v |v|^2 (masks: fixed dropout multipliers, or None)."""
    _, fm, x = deepfm(None, p, nd, dt, inputs=(dense, ids))
    layers = [(np.asarray(W, dt), np.asarray(b, dt)) for W, b in p["dnn_hidden"]] + \
             [(np.asarray(p["dnn_out"][0], dt), np.asarray(p["dnn_out"][1], dt))]
    acts = _dnn_train_acts(x, layers, "relu", masks, dt)
    dnn = acts[-1] @ layers[-1][0] + layers[-1][1]
    z = 0.5 * (fm + dnn)[:, 0]
    t = np.asarray(t, dt)
    ce = np.maximum(z, 0) - z * t + np.log1p(np.exp(-np.abs(z)))
    return np.mean(ce) + l2_w * np.sum(np.asarray(p["w1"], dt) ** 2) + l2_v * np.sum(np.asarray(p["v"], dt) ** 2)


def dcn_train_step(dense, ids, t, p, lr, reg_w, reg_b, nd=13, act="relu", dt=np.float64, masks=None):
    """One SGD step of compile_fit on DCN (model/dcn.py:24-34,
    utils/compile_fit.py:9-15), backpropagated by hand.  logit = [x_L | dnn]
    Wo + bo, g = (sigmoid(logit) - t)/B; CrossNet (layer/interaction.py:75-83)
    x_{l+1} = x0 g_l + b_l + x_l with g_l = x_l . w_l, backward
    delta_L = dL/dx_L, s_l = x0 . delta_{l+1}, dw_l = sum_b s_l x_l,
    db_l = sum_b delta_{l+1}, delta_l = delta_{l+1} + s_l w_l, dL/dx0 +=
    delta_0 + sum_l g_l delta_{l+1}; l2(reg) adds 2 reg w.  DNNLayer's
    Dropout: masks as in deepfm_train_step (None = the identity).  Returns
    (new p, losses before the step)."""
    dense = np.asarray(dense, dt)
    ids = cast_ids(ids)
    t = np.asarray(t, dt)
    tables = [np.array(tb, dt) for tb in p["tables"]]
    k = tables[0].shape[1]
    x = np.concatenate([dense, embed_layer(ids, tables, dt)], axis=1)
    B, d = x.shape
    ws = [np.array(w, dt).reshape(-1) for w in p["cross_w"]]
    bs = [np.array(b, dt).reshape(-1) for b in p["cross_b"]]
    xl, xs, gl = x, [x], []
    for w, b in zip(ws, bs):
        gl.append(xl @ w)
        xl = x * gl[-1][:, None] + b[None, :] + xl
        xs.append(xl)
    layers = [(np.array(W, dt), np.array(b, dt)) for W, b in p["dnn_hidden"]] + \
             [(np.array(p["dnn_out"][0], dt), np.array(p["dnn_out"][1], dt))]
    acts = _dnn_train_acts(x, layers, act, masks, dt)
    dnn = acts[-1] @ layers[-1][0] + layers[-1][1]
    z = np.concatenate([xl, dnn], axis=1)
    Wo, bo = np.array(p["out_kernel"], dt), np.array(p["out_bias"], dt)
    logit = (z @ Wo + bo)[:, 0]
    loss = np.maximum(logit, 0) - logit * t + np.log1p(np.exp(-np.abs(logit)))
    g = (sigmoid(logit) - t) / B
    dz = g[:, None] @ Wo.T
    out = {"out_kernel": Wo - lr * (z.T @ g[:, None]), "out_bias": bo - lr * g.sum(keepdims=True)}
    new_layers, dx = _dnn_train_bwd(dz[:, d:], layers, acts, act, masks, lr)
    dc = dz[:, :d]
    new_w, new_b = [None] * len(ws), [None] * len(ws)
    for l in reversed(range(len(ws))):
        s_l = np.sum(x * dc, axis=1)
        new_w[l] = (ws[l] - lr * (xs[l].T @ s_l + 2 * reg_w * ws[l])).reshape(-1, 1)
        new_b[l] = (bs[l] - lr * (dc.sum(0) + 2 * reg_b * bs[l])).reshape(-1, 1)
        dx = dx + gl[l][:, None] * dc
        dc = dc + s_l[:, None] * ws[l][None, :]
    dx = dx + dc
    out.update({"cross_w": new_w, "cross_b": new_b, "dnn_hidden": new_layers[:-1], "dnn_out": new_layers[-1]})
    for c, tb in enumerate(tables):
        np.add.at(tb, ids[:, c], -lr * dx[:, nd + c * k: nd + (c + 1) * k])
    out["tables"] = tables
    return out, loss


def dcn_loss(dense, ids, t, p, reg_w, reg_b, nd=13, dt=np.float64, masks=None):
    """compile_fit's objective on DCN: mean BCE(t, DCN.call) + reg_w sum |w_l|^2
    + reg_b sum |b_l|^2 (the Keras l2 regularisers); masks: fixed dropout
    multipliers of DNNLayer, or None."""
    q = dict(p, act=p.get("act", "relu"))
    x = np.concatenate([np.asarray(dense, dt), embed_layer(ids, p["tables"], dt)], axis=1)
    layers = [(np.asarray(W, dt), np.asarray(b, dt)) for W, b in p["dnn_hidden"]] + \
             [(np.asarray(p["dnn_out"][0], dt), np.asarray(p["dnn_out"][1], dt))]
    acts = _dnn_train_acts(x, layers, q["act"], masks, dt)
    z = np.concatenate([cross_layer(x, p["cross_w"], p["cross_b"], dt), acts[-1] @ layers[-1][0] + layers[-1][1]],
                       axis=1)
    logit = (z @ np.asarray(p["out_kernel"], dt) + np.asarray(p["out_bias"], dt))[:, 0]
    t = np.asarray(t, dt)
    ce = np.maximum(logit, 0) - logit * t + np.log1p(np.exp(-np.abs(logit)))
    return np.mean(ce) + reg_w * sum(np.sum(np.asarray(w, dt) ** 2) for w in p["cross_w"]) + \
        reg_b * sum(np.sum(np.asarray(b, dt) ** 2) for b in p["cross_b"])


def embed_fm_train_step(dense, ids, t, p, lr, l2_w, l2_v, nd=13, dt=np.float64):
    """One SGD step of compile_fit (utils/compile_fit.py:9-15) on
    sigmoid(FMLayer([dense | EmbedLayer(ids)])) — DeepFM's FM half
    (model/deepFM.py:23-31 without the DNN), the objective the row-sharded
    trainer (sharded.py train_step) optimises over its global batch:
    g = (sigmoid(fm) - t)/B; dx = g (w1 + v s - x |v|^2); dw1 = x^T g,
    dv = x^T (g s) - (x^2)^T g * v (+ 2 l2 terms), dw0 = sum g; rows by
    scatter-add.  p: {"tables", "w0", "w1", "v"}.  Returns (new p, losses)."""
    dense = np.asarray(dense, dt)
    ids = cast_ids(ids)
    t = np.asarray(t, dt)
    tables = [np.array(tb, dt) for tb in p["tables"]]
    k = tables[0].shape[1]
    x = np.concatenate([dense, embed_layer(ids, tables, dt)], axis=1)
    w0, w1, v = (np.array(p[n], dt) for n in ("w0", "w1", "v"))
    z = fm_layer(x, w0, w1, v, dt)[:, 0]
    loss = np.maximum(z, 0) - z * t + np.log1p(np.exp(-np.abs(z)))
    g = (sigmoid(z) - t) / x.shape[0]
    s = x @ v
    dx = g[:, None] * (w1[:, 0][None, :] + s @ v.T - x * np.sum(v * v, axis=1)[None, :])
    dw1 = x.T @ g[:, None]
    dv = x.T @ (g[:, None] * s) - ((x * x).T @ g)[:, None] * v
    out = {"w0": w0 - lr * g.sum(keepdims=True), "w1": w1 - lr * (dw1 + 2 * l2_w * w1),
           "v": v - lr * (dv + 2 * l2_v * v)}
    for c, tb in enumerate(tables):
        np.add.at(tb, ids[:, c], -lr * dx[:, nd + c * k: nd + (c + 1) * k])
    out["tables"] = tables
    return out, loss


def embed_fm_loss(dense, ids, t, p, l2_w, l2_v, nd=13, dt=np.float64):
    """Objective of embed_fm_train_step: mean BCE + l2_w |w1|^2 + l2_v |v|^2."""
    x = np.concatenate([np.asarray(dense, dt), embed_layer(ids, p["tables"], dt)], axis=1)
    z = fm_layer(x, p["w0"], p["w1"], p["v"], dt)[:, 0]
    t = np.asarray(t, dt)
    ce = np.maximum(z, 0) - z * t + np.log1p(np.exp(-np.abs(z)))
    return np.mean(ce) + l2_w * np.sum(np.asarray(p["w1"], dt) ** 2) + l2_v * np.sum(np.asarray(p["v"], dt) ** 2)
